// swim_oracle.cpp — CPU lockstep restatement of scalecube-cluster's protocol layer.
//
// TEST INFRASTRUCTURE ONLY.  This file is the parity oracle and the CPU baseline of bench.py.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
// (libswimgpu.so and the swimgpu package) never links, loads or falls back to it.
//
// It follows the reference Java line by line, with the sequential data structures the Java uses
// (ArrayList ping/remote lists, a TreeMap interval set per gossiper, an insertion-ordered gossip
// map, per-member tables), and fixes the canonical intra-tick order documented in DESIGN.md §3.
// Citations are to /root/reference/cluster/src/main/java/io/scalecube/cluster/ unless noted.
//
// Parity status: pinned by the reference's own known-answer tests (MembershipRecordTest,
// SequenceIdCollectorTest, ClusterMath values) and by scenario goldens restating
// FailureDetectorTest / MembershipProtocolTest / GossipProtocolTest outcomes (tests/).  The JVM
// reference itself cannot run here (no JDK), so the RNG-stream is defined by swim_rng.h, not by
// the JVM's ThreadLocalRandom.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "swim.h"
#include "swim_delay.h"
#include "swim_rng.h"

namespace {

constexpr uint32_t NONE = 0xffffffffu;

// ----------------------------------------------------------------------------- Philox4x32-10
void philox4x32_10(const uint32_t in[4], const uint32_t k[2], uint32_t out[4]) {
  uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
  uint32_t k0 = k[0], k1 = k[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

inline uint32_t next_int(uint32_t w, uint32_t bound) { return (uint32_t)(((uint64_t)w * bound) >> 32); }

// ----------------------------------------------------------------------------- records
enum Reason { FD_EVENT, MEMBERSHIP_GOSSIP, SYNC, INITIAL_SYNC, SUSPICION_TIMEOUT };  // :58-64

struct Record {  // MembershipRecord.java:20-22
  uint32_t member;
  uint32_t status;
  int32_t inc;
};

// MembershipRecord.isOverrides (MembershipRecord.java:67-88); r0 == nullptr for "no record".
bool is_overrides(const Record& r1, const Record* r0) {
  if (!r0) return r1.status == SWIM_ALIVE || r1.status == SWIM_LEAVING;
  if (r1.status == r0->status && r1.inc == r0->inc) return false;  // equals (member equal)
  if (r0->status == SWIM_DEAD) return false;
  if (r1.status == SWIM_DEAD) return true;
  if (r1.inc == r0->inc) return r1.status == SWIM_SUSPECT && (r0->status == SWIM_ALIVE || r0->status == SWIM_LEAVING);
  return r1.inc > r0->inc;
}

// A GET_METADATA round trip in flight under message delay (MetadataStoreImpl.fetchMetadata
// :146-185): stage 1 = the request travelling to the subject's address d, stage 2 = the response
// travelling back; `due` = the arrival tick of the current leg.  Draws stay keyed by the issue tick t0.
struct PendingFetch {
  uint32_t s;
  int32_t inc;
  uint32_t reason, phase, stage, f, d, ver;
  uint64_t t0, due;
  uint32_t link;  // the PendingAck (seq) whose Mono waits on this fetch, or NONE
};

// A merged message whose updateMembership Monos have not all completed (MembershipProtocolImpl.java
// syncMembership :491-509, Flux.mergeDelayError): onSync's SYNC_ACK waits for them (:394-415, the
// ack is prepared and sent in doOnSuccess), and so does start0's doFinally for an initial SYNC_ACK
// merged through its flatMap (:277-289).  A Mono waits on (a) an ALIVE admission's metadata fetch
// (:630-660 -> MetadataStoreImpl.fetchMetadata :146-185): a response ends it at its arrival, a failed
// send at once, anything unanswered at metadataTimeout; (b) a new LEAVING record's gossip
// (onLeavingDetected :710-733 returns spreadMembershipGossip, i.e. GossipProtocolImpl.spread's Mono,
// which completes when the gossip is most likely disseminated, :167-180 / :360-368).  Every other
// branch completes synchronously.
enum : uint32_t { PA_INITIAL_ACK = 1, PA_INIT = 2 };
struct PendingAck {
  uint32_t to;     // the SYNC's sender (the SYNC_ACK's receiver); PA_INIT: none
  uint32_t flags;  // PA_INITIAL_ACK: the SYNC was start0's (the ack goes to its Flux); PA_INIT: a start0 group
  uint32_t wn;     // fetches still in flight
  uint64_t ready;  // the tick the last completed / timed-out wait ended
  uint64_t gp;     // 1 + the infection period of the LEAVING gossips waited on (0: none)
  uint32_t seq;    // per member, in creation order (canonical order of the deferred acks)
};

// ----------------------------------------------------------------------------- SequenceIdCollector
// gossip/SequenceIdCollector.java:11-94 — closed intervals [a,b] in a TreeMap.
struct SeqCollector {
  // the TreeMap<Long, Long> of disjoint closed intervals [a, b] keyed by a, as a vector sorted by a
  // (a few intervals per collector: contiguous, 16 B each, where map nodes cost 64)
  std::vector<std::pair<int64_t, int64_t>> iv;
  // floorEntry(x): the last interval with a <= x, or -1
  ptrdiff_t floor_idx(int64_t x) const {
    auto it = std::upper_bound(iv.begin(), iv.end(), x,
                               [](int64_t v, const std::pair<int64_t, int64_t>& p) { return v < p.first; });
    return (it - iv.begin()) - 1;
  }
  // ceilingEntry(x): the first interval with a >= x (iv.size() if none)
  size_t ceil_idx(int64_t x) const {
    return (size_t)(std::lower_bound(iv.begin(), iv.end(), x,
                                     [](const std::pair<int64_t, int64_t>& p, int64_t v) { return p.first < v; }) -
                    iv.begin());
  }
  bool in_range(ptrdiff_t i, int64_t x) const { return i >= 0 && iv[i].first <= x && x <= iv[i].second; }
  bool next_to(ptrdiff_t i, int64_t x) const {
    return i >= 0 && (size_t)i < iv.size() && (x + 1 == iv[i].first || x - 1 == iv[i].second);
  }
  bool contains(int64_t x) const { return in_range(floor_idx(x), x); }  // :32-35
  bool add(int64_t x) {  // :43-72
    const ptrdiff_t fl = floor_idx(x);
    if (in_range(fl, x)) return false;
    const ptrdiff_t ce = (ptrdiff_t)ceil_idx(x);  // (fl + 1: x is in no interval)
    const bool nf = next_to(fl, x), nc = next_to(ce, x);
    if (nf && nc) {  // both neighbours: one interval [floor.a, ceiling.b]
      iv[fl].second = iv[ce].second;
      iv.erase(iv.begin() + ce);
    } else if (nf) {
      iv[fl].second = x;
    } else if (nc) {
      iv[ce].first = x;
    } else {
      iv.insert(iv.begin() + ce, {x, x});
    }
    return true;
  }
  size_t size() const { return iv.size(); }
  void clear() {
    iv.clear();
    iv.shrink_to_fit();
  }
};

// GossipState (gossip/GossipState.java:9-49) with its Gossip (Gossip.java, id = gossiper-seq)
// GossipState.infected, a HashSet<String> (GossipState.java:14), kept in insertion order: the first
// two members inline, the rest on the heap (almost every state holds one or two: no allocation)
struct InfSet {
  uint32_t a = 0xffffffffu, b = 0xffffffffu;
  std::vector<uint32_t>* more = nullptr;  // owned
  InfSet() = default;
  InfSet(const InfSet& o) : a(o.a), b(o.b), more(o.more ? new std::vector<uint32_t>(*o.more) : nullptr) {}
  InfSet(InfSet&& o) noexcept : a(o.a), b(o.b), more(o.more) { o.more = nullptr; }
  InfSet& operator=(InfSet o) noexcept {
    a = o.a;
    b = o.b;
    std::swap(more, o.more);
    return *this;
  }
  ~InfSet() { delete more; }
  size_t size() const { return (a != 0xffffffffu) + (b != 0xffffffffu) + (more ? more->size() : 0); }
  uint32_t operator[](size_t i) const { return i == 0 ? a : i == 1 ? b : (*more)[i - 2]; }
  bool contains(uint32_t m) const {
    return a == m || b == m || (more && std::find(more->begin(), more->end(), m) != more->end());
  }
  void push_back(uint32_t m) {
    if (a == 0xffffffffu) a = m;
    else if (b == 0xffffffffu) b = m;
    else {
      if (!more) more = new std::vector<uint32_t>();
      more->push_back(m);
    }
  }
};

// 40 B: the oracle keeps every live state of every member (config 3 at N = 4,096: ~4 x 10^8)
struct GossipState {
  uint32_t seq;               // Gossip.sequenceId (a member's own counter: < 2^32)
  uint32_t infection_period;  // GossipState.infectionPeriod (< 2^28, the engines' period bound)
  uint32_t gossiper;
  Record rec;
  InfSet infected;  // HashSet<String>, kept in insertion order
  bool is_infected(uint32_t m) const { return infected.contains(m); }
  void add_infected(uint32_t m) {
    if (!is_infected(m)) infected.push_back(m);
  }
};

// gossips.get(gossipId) (GossipProtocolImpl.java:206), the HashMap index of a member's gossip map:
// open addressing with linear probing and backward-shift deletion over 4-B slots, each the serial of
// a state (its insertion number: its position plus the states swept before it); a slot's key is
// read from the state itself (key_of)
struct GossipIndex {
  static constexpr uint32_t EMPTY = 0xffffffffu;
  std::vector<uint32_t> slot;
  size_t used = 0;
  static size_t hash(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return (size_t)x;
  }
  template <class KeyOf>
  void rehash(size_t cap, KeyOf key_of) {
    std::vector<uint32_t> old;
    old.swap(slot);
    slot.assign(cap, EMPTY);
    used = 0;
    for (uint32_t s : old)
      if (s != EMPTY) put(key_of(s), s, key_of);
  }
  template <class KeyOf>
  void put(uint64_t k, uint32_t s, KeyOf key_of) {
    if (2 * (used + 1) > slot.size()) rehash(std::max<size_t>(64, 2 * slot.size()), key_of);
    const size_t mask = slot.size() - 1;
    for (size_t i = hash(k) & mask;; i = (i + 1) & mask) {
      if (slot[i] == EMPTY) { slot[i] = s; ++used; return; }
      if (key_of(slot[i]) == k) { slot[i] = s; return; }
    }
  }
  template <class KeyOf>
  bool get(uint64_t k, uint32_t& s, KeyOf key_of) const {
    if (slot.empty()) return false;
    const size_t mask = slot.size() - 1;
    for (size_t i = hash(k) & mask;; i = (i + 1) & mask) {
      if (slot[i] == EMPTY) return false;
      if (key_of(slot[i]) == k) { s = slot[i]; return true; }
    }
  }
  template <class KeyOf>
  void erase(uint64_t k, KeyOf key_of) {
    if (slot.empty()) return;
    const size_t mask = slot.size() - 1;
    size_t i = hash(k) & mask;
    while (slot[i] == EMPTY || key_of(slot[i]) != k) {
      if (slot[i] == EMPTY) return;
      i = (i + 1) & mask;
    }
    // backward shift: move later entries of the run into the hole when their home allows it
    for (size_t j = (i + 1) & mask; slot[j] != EMPTY; j = (j + 1) & mask) {
      const size_t h = hash(key_of(slot[j])) & mask;
      if (((j - h) & mask) >= ((j - i) & mask)) {
        slot[i] = slot[j];
        i = j;
      }
    }
    slot[i] = EMPTY;
    --used;
  }
};

struct Member {
  bool up = false, joined = false, join_pending = false, join_now = false;
  // start0's initial sync (:250-291): requests sent / resolved (failed fast or answered), the tick
  // of the last answer (or of the start), and whether the merged Flux is still subscribed
  uint32_t init_total = 0, init_done = 0;
  uint64_t init_last = 0;
  bool init_wait = false;
  bool leave_pending = false, leave_done = false;
  uint32_t leave_gossiper = NONE;
  uint64_t leave_seq = 0;
  // ---- FailureDetectorImpl (:48-50)
  uint64_t fd_period = 0;
  std::vector<uint32_t> ping_members;
  uint32_t ping_index = 0;
  uint32_t ack_target = NONE;
  uint64_t ack_due = 0;
  bool ack_ok = false;    // ack_due is the tick the (delayed) ack arrives, not the timeout
  bool ack_gone = false;  // that ack says DEST_GONE (another member answers at the target's address)
  uint32_t ack_late = 0;  // 1 + ticks after the timeout that a late direct ack arrives (0 = none)
  uint64_t ack_to = 0;    // the ping's timeout tick (an ack dropped on arrival leaves the ping waiting)
  uint32_t relay_target = NONE, relay_pending = 0;
  uint64_t relay_due = 0;
  bool relay_ok = false;  // relay_due is the tick the first relayed ack arrives, not the timeout
  bool relay_gone = false;  // that ack says DEST_GONE
  uint32_t relay_first = NONE;  // the member that sent that ack (the issuer's inbound filter, on arrival)
  uint64_t relay_to = 0;  // the relay requests' timeout tick
  uint32_t join_addr = NONE;  // swim_join_at: the member whose address this joiner binds
  // ---- GossipProtocolImpl (:48-55)
  uint64_t g_period = 0, g_counter = 0, period_used = 0;
  std::unordered_map<uint32_t, SeqCollector> collectors;
  std::deque<GossipState> gossips;  // insertion order == canonical order
  GossipIndex gidx;                 // gossips.get(gossipId): id -> serial (HashMap lookup)
  uint32_t gbase = 0;               // serial of gossips.front() (states swept so far)
  uint32_t user_own = 0;            // own user gossips whose spread() has not completed
  // the first state in the spreading window (infectionPeriod + periodsToSpread >= period): infection
  // periods never decrease along the map, so the window is a suffix, found by binary search
  size_t window_start(uint64_t period, uint64_t spread) const {
    size_t lo = 0, hi = gossips.size();
    while (lo < hi) {
      const size_t mid = (lo + hi) / 2;
      if (gossips[mid].infection_period + spread >= period) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  }
  // (injective: gossiper < 2^24, seq < 2^32)
  static uint64_t gkey(uint32_t gossiper, uint64_t seq) { return ((uint64_t)gossiper << 40) ^ seq; }
  uint64_t key_at(uint32_t serial) const {
    const GossipState& g = gossips[serial - gbase];
    return gkey(g.gossiper, g.seq);
  }
  GossipState* find_gossip(uint32_t gossiper, uint64_t seq) {
    uint32_t s = 0;
    if (!gidx.get(gkey(gossiper, seq), s, [&](uint32_t x) { return key_at(x); })) return nullptr;
    return &gossips[s - gbase];
  }
  void add_gossip(const GossipState& g) {
    if (gbase + gossips.size() >= 0xffffffffull) std::abort();  // (serials are 32-bit)
    gossips.push_back(g);
    const uint32_t s = gbase + (uint32_t)gossips.size() - 1;
    gidx.put(gkey(g.gossiper, g.seq), s, [&](uint32_t x) { return key_at(x); });
  }
  // the sweep (:158-164, :350-358) drops the states with period > infectionPeriod + sweep.  Infection
  // periods never decrease along the map (a state takes its holder's current period when it is
  // added), so those are a prefix: dropped from the front, the index loses their keys only
  void sweep_gossips(uint64_t period, uint64_t sweep) {
    size_t p0 = 0;
    while (p0 < gossips.size() && period > gossips[p0].infection_period + sweep) ++p0;
    for (size_t i = p0; i < gossips.size(); ++i)
      if (period > gossips[i].infection_period + sweep) std::abort();  // (not a prefix: impossible)
    for (size_t i = 0; i < p0; ++i)  // (the keys leave the index while their states still exist)
      gidx.erase(key_at(gbase + (uint32_t)i), [&](uint32_t x) { return key_at(x); });
    for (size_t i = 0; i < p0; ++i) gossips.pop_front();
    gbase += (uint32_t)p0;
  }
  std::vector<uint32_t> remote;
  int32_t remote_index = -1;
  // ---- MembershipProtocolImpl: table / members / aliveEmittedSet / metadata / timers live in
  // the packed row (swim.h cell format), one word per subject.
  std::vector<uint64_t> row;
  uint32_t table_size = 0, members_size = 0;
  std::vector<uint32_t> fd_sync;  // SYNCs requested by FD ALIVE events this tick (:427-442)
  // timer phases
  int64_t fd_start = 0, g_start = 0, sync_start = 0;
  bool sync_on = false;
  // per-tick bookkeeping
  uint32_t ev_minor = 0, fetch_ctr = 0;
  std::vector<PendingFetch> fq;  // metadata round trips in flight, in issue order
  // deferred SYNC_ACKs and start0 groups (PendingAck), in creation order; the waits of the message
  // being merged (w_link = the seq its PendingAck will take, NONE outside such a merge)
  std::vector<PendingAck> pack;
  uint32_t pack_seq = 0, init_pend = 0;
  // this member's own MembershipConfig.seedMembers (swim_set_member_seeds), else the engine-wide list
  bool own_seeds = false;
  std::vector<uint32_t> seeds;
  uint32_t w_link = NONE, w_n = 0;
  uint64_t w_ready = 0, w_gp = 0;
  uint64_t ctl_tick1 = 0;  // 1 + the tick of the member's last control-phase operation (swim_ingest_sync)
};

// cell helpers
constexpr uint64_t B_IN_TABLE = 1ull << 34, B_IN_MEMBERS = 1ull << 35, B_ALIVE_EMITTED = 1ull << 36,
                   B_HAS_TIMER = 1ull << 37, B_HAS_METADATA = 1ull << 38;
inline int32_t c_inc(uint64_t c) { return (int32_t)(uint32_t)c; }
inline uint32_t c_status(uint64_t c) { return (uint32_t)((c >> 32) & 3u); }
inline bool c_has(uint64_t c, uint64_t bit) { return (c & bit) != 0; }
inline uint32_t c_deadline(uint64_t c) { return (uint32_t)(c >> 39); }
inline uint64_t c_with_record(uint64_t c, uint32_t status, int32_t inc) {
  return (c & ~0x3ffffffffull) | (uint64_t)(uint32_t)inc | ((uint64_t)status << 32);
}
inline uint64_t c_with_deadline(uint64_t c, uint64_t tick) {
  return (c & ((1ull << 39) - 1)) | ((tick & SWIM_DEADLINE_MASK) << 39);
}

struct LinkKey {
  uint32_t a, b;
  bool operator<(const LinkKey& o) const { return a < o.a || (a == o.a && b < o.b); }
};

struct SyncReq {
  uint32_t from, to, ordinal;
  bool initial, outfail, delivered, acked;
};

struct PendingAlive {
  Record r1;
};


// Side effects a worker thread of a parallel phase region collects instead of writing the engine's
// shared stats / event list / timer queue; merged in thread order after the region (the CPU
// baseline's multi-threaded mode, swim_oracle_set_threads).  Every other write of a phase touches
// only the state of the member the worker owns in that phase.
struct Acc {
  swim_stats st{};
  std::vector<swim_event> ev;
  std::vector<std::pair<uint64_t, std::pair<uint32_t, uint32_t>>> timers;
};
thread_local Acc* tl_acc = nullptr;

}  // namespace

struct swim_engine {
  swim_config cfg{};
  uint32_t n = 0;
  uint64_t seed = 0;
  uint32_t key[2]{};
  uint64_t T = 0;
  uint32_t tick_ms = 0, P = 0, to_ticks = 0, relay_ticks = 0, G = 0, S = 0, sync_to_ticks = 0;
  uint32_t mt_ticks = 0;  // ceil(metadataTimeout / tick): an unanswered fetch fails this many ticks after it was sent
  std::vector<Member> m;
  std::vector<uint32_t> seeds;
  std::vector<uint8_t> is_seed;
  // addresses (swim_join_at): addr[x] = the address member x was started on (a slot number),
  // route[x] = the member whose transport listens on x's address now; both empty while every member
  // is on its own address
  std::vector<uint32_t> addr, route;
  // network emulator
  std::vector<int32_t> default_loss;
  std::vector<uint8_t> default_inbound;
  std::map<LinkKey, int32_t> link_loss;     // (src,dst) -> loss %
  std::map<LinkKey, uint8_t> link_inbound;  // (dst,src) -> shallPass
  // MembershipConfig.namespace of each member as a group id, and which groups are related
  // (areNamespacesRelated :511-536); n_ns = 0: one namespace
  std::vector<uint16_t> ns;
  std::vector<uint8_t> ns_rel;
  uint32_t n_ns = 0;
  // metadata: version of each member's metadata (ClusterImpl.updateMetadata :497-500 bumps it) and,
  // once a metadata update happened, the version each viewer's MetadataStore holds per subject
  std::vector<uint32_t> meta_ver;
  std::vector<std::vector<uint32_t>> meta_seen;
  std::vector<int32_t> default_delay;       // OutboundSettings.meanDelay (ms) per member
  std::map<LinkKey, int32_t> link_delay;    // (src,dst) -> meanDelay (ms)
  std::map<int32_t, std::vector<uint64_t>> delay_tab;  // meanDelay -> thresholds (swim_delay.h)
  // GOSSIP_REQs in flight: arrival tick -> messages (sent in an earlier tick's gossip round)
  struct DelayedMsg {
    uint32_t to, from, pos;
    uint64_t sent;
  };
  bool partition = false;
  std::vector<uint16_t> group;
  // timers: deadline tick -> (viewer, subject)
  std::map<uint64_t, std::vector<std::pair<uint32_t, uint32_t>>> timer_queue;
  std::vector<swim_event> events;
  swim_stats st{};
  uint32_t threads = 1;  // worker threads of the per-member phase loops (1 = the plain sequential loops)

  swim_stats& STT() { return tl_acc ? tl_acc->st : st; }

  // fn(a, b, t) over [lo, hi) split into `threads` contiguous ranges (t = range index), one
  // std::thread each, then the workers' side effects merged in range order
  template <class F>
  void par(uint32_t lo, uint32_t hi, F&& fn) {
    const uint32_t nt = threads;
    if (nt <= 1 || hi - lo < 2 * nt) {
      fn(lo, hi, 0u);
      return;
    }
    std::vector<Acc> acc(nt);
    std::vector<std::thread> th;
    th.reserve(nt);
    for (uint32_t t = 0; t < nt; ++t) {
      const uint32_t a = lo + (uint32_t)((uint64_t)(hi - lo) * t / nt);
      const uint32_t b = lo + (uint32_t)((uint64_t)(hi - lo) * (t + 1) / nt);
      th.emplace_back([&, a, b, t] {
        tl_acc = &acc[t];
        fn(a, b, t);
        tl_acc = nullptr;
      });
    }
    for (auto& x : th) x.join();
    for (auto& a : acc) {
      uint64_t* d = reinterpret_cast<uint64_t*>(&st);
      const uint64_t* x = reinterpret_cast<const uint64_t*>(&a.st);
      for (size_t i = 0; i < sizeof(swim_stats) / 8; ++i) d[i] += x[i];
      events.insert(events.end(), a.ev.begin(), a.ev.end());
      for (auto& tq : a.timers) timer_queue[tq.first].push_back(tq.second);
    }
  }

  // ------------------------------------------------------------------------- RNG
  uint32_t draw(uint32_t member, uint32_t stream, uint32_t sub24, uint32_t sub32, uint64_t tick) const {
    uint32_t c[4] = {member, (uint32_t)tick, (stream << 24) | (sub24 & 0xffffffu), sub32};
    uint32_t o[4];
    philox4x32_10(c, key, o);
    return o[0];
  }
  uint32_t draw(uint32_t member, uint32_t stream, uint32_t sub24, uint32_t sub32) const {
    return draw(member, stream, sub24, sub32, T);
  }
  static bool lost(int32_t pct, uint32_t w) { return pct > 0 && (pct >= 100 || (int32_t)next_int(w, 100) < pct); }

  // ------------------------------------------------------------------------- addresses
  // the member a message sent to x's address reaches (Transport.send / requestResponse by Address)
  uint32_t dst(uint32_t x) const { return route.empty() ? x : route[x]; }
  // member m starts listening on the address of member a (whose transport is stopped)
  void bind_address(uint32_t m_, uint32_t a) {
    if (route.empty()) {
      route.resize(n);
      addr.resize(n);
      for (uint32_t x = 0; x < n; ++x) route[x] = addr[x] = x;
    }
    const uint32_t A = addr[a];
    addr[m_] = A;
    for (uint32_t x = 0; x < n; ++x)
      if (addr[x] == A) route[x] = m_;
  }

  // ------------------------------------------------------------------------- NetworkEmulator
  // OutboundSettings resolution (NetworkEmulator.java:59-61), partition shorthand first.
  int32_t out_loss(uint32_t a, uint32_t b) const {
    if (partition && group[a] != group[b]) return 100;
    auto it = link_loss.find({a, b});
    if (it != link_loss.end()) return it->second;
    return default_loss[a];
  }
  // InboundSettings of receiver b for sender a (NetworkEmulator.java:212-214)
  bool in_pass(uint32_t b, uint32_t a) const {
    auto it = link_inbound.find({b, a});
    if (it != link_inbound.end()) return it->second != 0;
    return default_inbound[b] != 0;
  }
  // tryFailOutbound (:167-181) + a stopped destination refusing the connection
  bool out_fail(uint32_t a, uint32_t b, uint32_t w) const { return !m[b].up || lost(out_loss(a, b), w); }
  // tryDelayOutbound (:190-202) + evaluateDelay (:359-369), in ticks (swim_delay.h); the draw is
  // keyed (member, stream, sub24, sub32) and taken only when the link has a mean delay
  int32_t out_delay(uint32_t a, uint32_t b) const {
    auto it = link_delay.find({a, b});
    return it != link_delay.end() ? it->second : default_delay[a];
  }
  uint32_t delay_ticks(uint32_t a, uint32_t b, uint32_t member, uint32_t stream, uint32_t sub24, uint32_t sub32) {
    return delay_ticks_at(a, b, member, stream, sub24, sub32, T);
  }
  uint32_t delay_ticks_at(uint32_t a, uint32_t b, uint32_t member, uint32_t stream, uint32_t sub24, uint32_t sub32,
                          uint64_t tick) {
    const int32_t mean = out_delay(a, b);
    if (mean <= 0) return 0;
    uint32_t c[4] = {member, (uint32_t)tick, (stream << 24) | (sub24 & 0xffffffu), sub32}, o[4];
    philox4x32_10(c, key, o);
    const uint64_t u53 = ((uint64_t)(o[0] >> 11) << 32) | o[1];
    return swim_delay_ticks(delay_tab.at(mean).data(), u53);
  }
  // a mean the engine refuses changes nothing (swim_delay_mean_ok; at most 4,096 distinct means, the
  // GPU engine's delay-table limit)
  bool delay_mean_acceptable(int32_t mean) const {
    return swim_delay_mean_ok(mean, tick_ms) && (delay_tab.count(mean) || delay_tab.size() < 4096);
  }
  void ensure_delay_tab(int32_t mean) {
    if (mean <= 0 || delay_tab.count(mean)) return;
    std::vector<uint64_t> th(SWIM_DELAY_TICKS_MAX);
    swim_delay_thresholds(mean, tick_ms, th.data());
    delay_tab[mean] = std::move(th);
  }

  // ------------------------------------------------------------------------- events
  void emit(uint32_t v, uint32_t subject, uint32_t type, uint32_t phase, uint32_t minor, uint32_t data = 0) {
    swim_event e{};
    e.data = data;
    e.tick = T;
    e.viewer = v;
    e.subject = subject;
    e.type = type;
    e.phase = phase;
    e.minor = minor;
    if (tl_acc) tl_acc->ev.push_back(e); else events.push_back(e);
    STT().events++;
  }
  uint32_t next_minor(uint32_t v) { return m[v].ev_minor++; }

  // FailureDetectorImpl.onMemberEvent (:321-346) + GossipProtocolImpl.onMemberEvent (:238-261)
  void on_member_added(uint32_t v, uint32_t s, uint32_t phase, uint32_t minor) {
    auto& pm = m[v].ping_members;
    uint32_t size = (uint32_t)pm.size();
    uint32_t idx = size > 0 ? next_int(draw(v, SWIM_STREAM_PING_INSERT, phase, minor), size) : 0;
    pm.insert(pm.begin() + idx, s);
    m[v].remote.push_back(s);
  }
  void on_member_removed(uint32_t v, uint32_t s) {
    auto& pm = m[v].ping_members;
    auto it = std::find(pm.begin(), pm.end(), s);
    if (it != pm.end()) pm.erase(it);
    auto& rm = m[v].remote;
    auto it2 = std::find(rm.begin(), rm.end(), s);
    if (it2 != rm.end()) rm.erase(it2);
    m[v].collectors.erase(s);  // sequenceIdCollectors.remove(member.id()) (:242)
  }
  void publish_event(uint32_t v, uint32_t s, uint32_t type, uint32_t phase, uint32_t minor) {
    emit(v, s, type, phase, minor);
    if (type == SWIM_EV_ADDED) on_member_added(v, s, phase, minor);
    if (type == SWIM_EV_REMOVED) on_member_removed(v, s);
  }
  uint32_t ev_minor_for(uint32_t v, uint32_t phase, uint32_t subject) {
    return phase == SWIM_PHASE_TIMERS ? subject : next_minor(v);
  }

  // ------------------------------------------------------------------------- gossip origination
  // spreadMembershipGossip (MembershipProtocolImpl.java:845-860) -> GossipProtocolImpl.spread ->
  // createAndPutGossip (GossipProtocolImpl.java:190-199)
  // `why`: the call site (SWIM_ORIG_*), counted in swim_stats.gossips_by_reason
  void spread_gossip(uint32_t v, const Record& r, uint32_t why) {
    Member& mv = m[v];
    GossipState g;
    g.gossiper = v;
    g.seq = (uint32_t)mv.g_counter++;
    g.rec = r;
    g.infection_period = (uint32_t)mv.g_period;
    mv.add_gossip(g);
    mv.collectors[v].add((int64_t)g.seq);
    STT().gossips_created++;
    STT().gossips_by_reason[why]++;
  }
  // the SWIM_ORIG_* reason of a spreadMembershipGossipUnlessGossiped call (:836-843)
  static uint32_t orig_of(Reason r) { return r == FD_EVENT ? SWIM_ORIG_FD : SWIM_ORIG_SYNC; }

  // GossipProtocol.spread(Message) (GossipProtocolImpl.java:126-130): a user gossip, its payload in
  // the record's member field (status SWIM_GOSSIP_USER)
  void spread_user(uint32_t v, uint32_t payload) {
    spread_gossip(v, Record{payload, SWIM_GOSSIP_USER, 0}, SWIM_ORIG_USER);
    m[v].user_own++;
  }

  // ------------------------------------------------------------------------- timers
  // scheduleSuspicionTimeoutTask (:805-823): computeIfAbsent, timeout from the table size now.
  void schedule_timer(uint32_t v, uint32_t s) {
    uint64_t& c = m[v].row[s];
    if (c_has(c, B_HAS_TIMER)) return;
    int64_t ms = swim_suspicion_timeout(cfg.suspicion_mult, (int32_t)m[v].table_size, cfg.ping_interval);
    uint64_t deadline = T + (uint64_t)(ms / tick_ms);
    c = c_with_deadline(c | B_HAS_TIMER, deadline);
    if (tl_acc) tl_acc->timers.push_back({deadline, {v, s}}); else timer_queue[deadline].push_back({v, s});
  }
  // cancelSuspicionTimeoutTask (:797-803)
  void cancel_timer(uint32_t v, uint32_t s) { m[v].row[s] &= ~B_HAS_TIMER; }

  // ------------------------------------------------------------------------- metadata fetch
  // MetadataStoreImpl.fetchMetadata (:146-185) round trip + onMetadataRequest (:201-240), with the
  // NetworkEmulator's arrival-time semantics: the request is lost or refused at its send, meets the
  // subject's transport (stopped, inbound filter) when it arrives; the response likewise; the whole
  // round trip must end before metadataTimeout (:160-165).  Returns true when the response is in
  // within the calling phase (no delay on either leg: the caller applies the admission at its flush
  // point); a delayed round trip goes to the viewer's queue and completes in the FETCH phase of its
  // arrival tick (phase_fetch).
  bool fetch_start(uint32_t v, const Record& r1, Reason reason, uint32_t phase) {
    Member& mv = m[v];
    const uint32_t f = mv.fetch_ctr++;
    STT().fetches++;
    const uint32_t s = r1.member, d = dst(s);
    // an unanswered request fails at metadataTimeout (:160-165): a Mono waiting on it ends then
    auto timeout = [&] { if (mv.w_link != NONE) mv.w_ready = std::max(mv.w_ready, T + mt_ticks); };
    // the request goes to s's address; another member listening there does not answer (:209)
    if (d != s) { timeout(); return false; }
    if (out_fail(v, d, draw(v, SWIM_STREAM_FETCH_REQ, phase, f))) return false;  // fails at once
    const uint32_t d1 = delay_tab.empty() ? 0 : delay_ticks(v, d, v, SWIM_STREAM_FETCH_REQ_DELAY, phase, f);
    if ((uint64_t)d1 * tick_ms >= (uint64_t)cfg.metadata_timeout) { timeout(); return false; }
    PendingFetch p{s, r1.inc, (uint32_t)reason, phase, 1, f, d, 0, T, T + d1, mv.w_link};
    if (d1 == 0) {
      const int r = fetch_stage1(v, p);
      if (r == 1) STT().fetch_ok++;
      if (r == 0) timeout();
      if (r != 2) return r == 1;
    }
    if (mv.w_link != NONE) mv.w_n++;
    mv.fq.push_back(p);
    return false;
  }
  // the PendingAck of member v with sequence number seq (nullptr: none — cancelled with start0's Flux)
  PendingAck* pack_find(uint32_t v, uint32_t seq) {
    for (auto& a : m[v].pack)
      if (a.seq == seq) return &a;
    return nullptr;
  }
  // a message's merge starts / ends: its waits are collected, and a message whose Monos have not all
  // completed by now becomes a PendingAck (returns true: the SYNC_ACK waits)
  void wait_begin(uint32_t v) {
    Member& mv = m[v];
    mv.w_link = mv.pack_seq;
    mv.w_n = 0;
    mv.w_ready = 0;
    mv.w_gp = 0;
  }
  bool wait_end(uint32_t v, uint32_t to, uint32_t flags) {
    Member& mv = m[v];
    mv.w_link = NONE;
    if (mv.w_n == 0 && mv.w_gp == 0 && mv.w_ready <= T) return false;
    mv.pack.push_back(PendingAck{to, flags, mv.w_n, mv.w_ready, mv.w_gp, mv.pack_seq++});
    if (flags & PA_INIT) mv.init_pend++;
    return true;
  }
  // the request arrives at d (now): 0 = the round trip failed, 1 = the response arrived too (no delay
  // on it), 2 = the response is in flight (p.due = its arrival tick)
  int fetch_stage1(uint32_t v, PendingFetch& p) {
    const uint32_t d = p.d;
    if (!m[d].up || !in_pass(d, v)) return 0;
    if (out_fail(d, v, draw(v, SWIM_STREAM_FETCH_RESP, p.phase, p.f, p.t0))) return 0;
    const uint32_t d2 =
        delay_tab.empty() ? 0 : delay_ticks_at(d, v, v, SWIM_STREAM_FETCH_RESP_DELAY, p.phase, p.f, p.t0);
    if ((T - p.t0 + d2) * tick_ms >= (uint64_t)cfg.metadata_timeout) return 0;
    p.ver = meta_ver.empty() ? 0 : meta_ver[p.s];  // the metadata the response carries
    p.stage = 2;
    p.due = T + d2;
    if (d2 == 0) return fetch_stage2(v, p) ? 1 : 0;
    return 2;
  }
  // the response arrives at v (now)
  bool fetch_stage2(uint32_t v, const PendingFetch& p) const { return m[v].up && in_pass(v, p.d); }

  // ------------------------------------------------------------------------- updateMembership
  // MembershipProtocolImpl.updateMembership (:569-664).  ALIVE admissions whose metadata fetch
  // succeeds are appended to `pending` and applied by apply_alive at the caller's flush point.
  void update_membership(uint32_t v, const Record& r1, Reason reason, uint32_t phase,
                         std::vector<PendingAlive>& pending) {
    Member& mv = m[v];
    const uint32_t s = r1.member;
    uint64_t& c = mv.row[s];
    // namespace filter (:575-586)
    if (n_ns && !ns_rel[(size_t)ns[v] * n_ns + ns[s]]) return;
    const bool present = c_has(c, B_IN_TABLE);
    Record r0v{s, c_status(c), c_inc(c)};
    const Record* r0 = present ? &r0v : nullptr;
    const bool r0_leaving = present && r0v.status == SWIM_LEAVING;
    if (!r0_leaving && !is_overrides(r1, r0)) return;  // :593-602

    if (s == v) {  // onSelfMemberDetected (:686-708)
      int32_t cur = std::max(r0v.inc, r1.inc);
      Record r2{v, r0v.status, cur + 1};
      c = c_with_record(c, r2.status, r2.inc);
      spread_gossip(v, r2, SWIM_ORIG_REFUTE);
      return;
    }
    if (dst(s) == v) return;  // another member at the local address (:605-610)
    if (r1.status == SWIM_LEAVING) {  // onLeavingDetected (:710-733)
      if (!present) { mv.table_size++; }
      c = c_with_record(c | B_IN_TABLE, SWIM_LEAVING, r1.inc);
      if (present && (r0v.status == SWIM_ALIVE ||
                      (r0v.status == SWIM_SUSPECT && c_has(c, B_ALIVE_EMITTED)))) {
        publish_event(v, s, SWIM_EV_LEAVING, phase, ev_minor_for(v, phase, s));
      }
      if (!present || r0v.status != SWIM_LEAVING) {
        schedule_timer(v, s);
        spread_gossip(v, r1, SWIM_ORIG_LEAVING);
        // onLeavingDetected returns the gossip's spread() Mono: a merge waits until it disseminated
        if (mv.w_link != NONE) mv.w_gp = mv.g_period + 1;
      }
      return;
    }
    if (r1.status == SWIM_DEAD) {  // onDeadMemberDetected (:740-767)
      cancel_timer(v, s);
      if (!c_has(c, B_IN_MEMBERS)) return;
      c = 0;
      mv.table_size--;
      mv.members_size--;
      publish_event(v, s, SWIM_EV_REMOVED, phase, ev_minor_for(v, phase, s));
      return;
    }
    if (r1.status == SWIM_SUSPECT) {  // :621-628
      if (!r0_leaving) {
        if (!present) mv.table_size++;  // unreachable: SUSPECT never overrides a missing row
        c = c_with_record(c | B_IN_TABLE, SWIM_SUSPECT, r1.inc);
      }
      schedule_timer(v, s);
      if (reason != MEMBERSHIP_GOSSIP && reason != INITIAL_SYNC) spread_gossip(v, r1, orig_of(reason));
      return;
    }
    // ALIVE (:630-660)
    if (r0_leaving) {  // onAliveAfterLeaving (:666-684)
      if (!c_has(c, B_IN_MEMBERS)) { c |= B_IN_MEMBERS; mv.members_size++; }
      if (!c_has(c, B_ALIVE_EMITTED)) {
        c |= B_ALIVE_EMITTED;
        publish_event(v, s, SWIM_EV_ADDED, phase, ev_minor_for(v, phase, s));
        publish_event(v, s, SWIM_EV_LEAVING, phase, ev_minor_for(v, phase, s));
      }
      return;
    }
    if (!present || r0v.inc < r1.inc) {
      if (fetch_start(v, r1, reason, phase)) pending.push_back(PendingAlive{r1});
    }
  }

  // doOnSuccess of the fetch (:648-656) + onAliveMemberDetected (:769-795)
  void apply_alive(uint32_t v, const Record& r1, Reason reason, uint32_t phase) {
    apply_alive(v, r1, reason, phase, meta_ver.empty() ? 0 : meta_ver[r1.member]);
  }
  // ver: the subject's metadata version the response carried
  void apply_alive(uint32_t v, const Record& r1, Reason reason, uint32_t phase, uint32_t ver) {
    Member& mv = m[v];
    const uint32_t s = r1.member;
    cancel_timer(v, s);
    if (reason != MEMBERSHIP_GOSSIP && reason != INITIAL_SYNC) spread_gossip(v, r1, orig_of(reason));
    uint64_t& c = mv.row[s];
    // metadataStore.updateMetadata(member, metadata1) returns metadata0 (null when none is stored);
    // metadata1 is the subject's metadata when it answered
    const bool had_meta = c_has(c, B_HAS_METADATA);
    bool same_meta = had_meta;
    if (!meta_seen.empty()) {
      same_meta = had_meta && meta_seen[v][s] == ver;
      meta_seen[v][s] = ver;
    }
    c |= B_HAS_METADATA;
    const bool exists = c_has(c, B_IN_MEMBERS);
    if (!c_has(c, B_IN_TABLE)) mv.table_size++;
    if (!exists) mv.members_size++;
    c = c_with_record(c | B_IN_TABLE | B_IN_MEMBERS, SWIM_ALIVE, r1.inc);
    if (!exists) {
      publish_event(v, s, SWIM_EV_ADDED, phase, ev_minor_for(v, phase, s));
      c |= B_ALIVE_EMITTED;
    } else if (!same_meta) {  // !metadata1.equals(metadata0) (:780-781)
      publish_event(v, s, SWIM_EV_UPDATED, phase, ev_minor_for(v, phase, s));
    }
  }

  void flush_pending(uint32_t v, std::vector<PendingAlive>& pending, Reason reason, uint32_t phase) {
    for (auto& p : pending) apply_alive(v, p.r1, reason, phase);
    pending.clear();
  }

  // ------------------------------------------------------------------------- phase A: timers
  // onSuspicionTimeout (:825-834), due (viewer, subject) pairs in ascending order.
  void phase_timers() {
    auto it = timer_queue.find(T);
    if (it == timer_queue.end()) return;
    auto due = std::move(it->second);
    timer_queue.erase(it);
    std::sort(due.begin(), due.end());
    due.erase(std::unique(due.begin(), due.end()), due.end());
    // a worker owns the viewers of its range: their due entries are one stretch of the sorted list
    par(0, n, [&](uint32_t va, uint32_t vb, uint32_t) {
      std::vector<PendingAlive> none;
      auto it = std::lower_bound(due.begin(), due.end(), std::make_pair(va, 0u));
      for (; it != due.end() && it->first < vb; ++it) {
        uint32_t v = it->first, s = it->second;
        if (!m[v].up) continue;
        uint64_t& c = m[v].row[s];
        if (!c_has(c, B_HAS_TIMER) || c_deadline(c) != (uint32_t)(T & SWIM_DEADLINE_MASK)) continue;
        c &= ~B_HAS_TIMER;
        STT().timers_fired++;
        if (c_has(c, B_IN_TABLE)) {
          Record dead{s, SWIM_DEAD, c_inc(c)};
          update_membership(v, dead, SUSPICION_TIMEOUT, SWIM_PHASE_TIMERS, none);
        }
      }
    });
  }

  // ------------------------------------------------------------------------- phase B: FD
  // publishPingResult (:377-380) -> MembershipProtocolImpl.onFailureDetectorEvent (:418-449)
  void publish_fd(uint32_t v, uint32_t t, uint32_t status) {
    STT().fd_events++;
    if (cfg.record_fd_events)
      emit(v, t, SWIM_EV_FD_ALIVE + (status == SWIM_ALIVE ? 0 : status == SWIM_SUSPECT ? 1 : 2),
           SWIM_PHASE_FD, next_minor(v));
    uint64_t c = m[v].row[t];
    if (!c_has(c, B_IN_TABLE)) return;
    if (c_status(c) == status) return;
    if (status == SWIM_ALIVE) {
      m[v].fd_sync.push_back(t);
      return;
    }
    std::vector<PendingAlive> none;
    update_membership(v, Record{t, status, c_inc(c)}, FD_EVENT, SWIM_PHASE_FD, none);
  }

  // Collections.shuffle (for i = size; i > 1; i--) swap(i-1, nextInt(i))
  void shuffle(uint32_t v, std::vector<uint32_t>& list, uint32_t stream) {
    for (uint32_t i = (uint32_t)list.size(); i > 1; --i) {
      uint32_t j = next_int(draw(v, stream, 0, i), i);
      std::swap(list[i - 1], list[j]);
    }
  }

  // selectPingMember (:352-361)
  uint32_t select_ping_member(uint32_t v) {
    auto& pm = m[v].ping_members;
    if (pm.empty()) return NONE;
    if (m[v].ping_index >= pm.size()) {
      m[v].ping_index = 0;
      shuffle(v, pm, SWIM_STREAM_FD_SHUFFLE);
    }
    return pm[m[v].ping_index++];
  }

  // selectPingReqMembers (:363-375): uniformly random ordered k-subset of pingMembers \ {target},
  // drawn by a forward partial Fisher-Yates over the candidate positions.
  std::vector<uint32_t> select_ping_req_members(uint32_t v, uint32_t t) {
    std::vector<uint32_t> out;
    const int32_t k = cfg.ping_req_members;
    if (k <= 0) return out;
    const auto& pm = m[v].ping_members;
    int64_t pos = -1;
    for (size_t i = 0; i < pm.size(); ++i)
      if (pm[i] == t) { pos = (int64_t)i; break; }
    const uint32_t cnt = (uint32_t)pm.size() - (pos >= 0 ? 1u : 0u);
    if (cnt == 0) return out;
    const uint32_t r = std::min<uint32_t>((uint32_t)k, cnt);
    std::vector<std::pair<uint32_t, uint32_t>> sw;  // sparse position -> value
    auto get = [&](uint32_t p) {
      for (auto& e : sw) if (e.first == p) return e.second;
      return p;
    };
    auto set = [&](uint32_t p, uint32_t val) {
      for (auto& e : sw) if (e.first == p) { e.second = val; return; }
      sw.push_back({p, val});
    };
    for (uint32_t i = 0; i < r; ++i) {
      uint32_t j = i + next_int(draw(v, SWIM_STREAM_RELAY_SELECT, i, 0), cnt - i);
      uint32_t vi = get(i), vj = get(j);
      set(i, vj);
      set(j, vi);
      uint32_t x = vj;
      out.push_back((pos >= 0 && (int64_t)x >= pos) ? pm[x + 1] : pm[x]);
    }
    return out;
  }

  // doPing's error branch (:153-170) + doPingReq (:173-210).  Every pending relay request shares
  // the ping's correlation id, so the first relayed ack that reaches the issuer completes all of
  // them (TransportImpl.requestResponse :214-238 filters listen() by cid only).
  // With message delay the first message carrying the cid to arrive decides: the earliest relayed
  // ack (ties: lowest relay), or a late ack of the direct ping (`late` = 1 + its arrival in ticks
  // after the ping-req went out, 0 = none; it carries the same cid and arrives after the relay
  // requests subscribed), and only if the issuer's inbound filter passes its sender
  // (NetworkEmulatorTransport.requestResponse :65-74, applied when that message ARRIVES: each
  // requestResponse takes the first message with its cid and drops it there if the filter blocks it,
  // so a blocked first ack completes none of them); none before pingInterval - pingTimeout: SUSPECT.
  // Every message goes to an address (dst): a relay's transit ping reaches whoever listens at t's
  // address, and that member's onPing answers DEST_GONE when it is not t (:227-259), which every
  // ack carries back (onTransitPingAck :291-315) and computeMemberStatus turns into DEAD (:382-404).
  void ping_req(uint32_t v, uint32_t t, uint32_t late = 0, bool late_gone = false) {
    std::vector<uint32_t> relays = select_ping_req_members(v, t);
    if (relays.empty()) {  // timeLeft <= 0 is excluded by config validation
      publish_fd(v, t, SWIM_SUSPECT);
      return;
    }
    STT().ping_reqs++;
    std::vector<uint32_t> pending;
    const uint32_t d = dst(t);
    const bool gone = d != t;
    for (uint32_t j = 0; j < relays.size(); ++j) {
      if (out_fail(v, dst(relays[j]), draw(v, SWIM_STREAM_PINGREQ_OUT, j, 0)))
        publish_fd(v, t, SWIM_SUSPECT);  // immediate outbound error
      else
        pending.push_back(j);
    }
    if (pending.empty()) return;
    uint32_t best = NONE, first = NONE;  // arrival (ticks after now) and sender of the first ack
    bool first_gone = gone;
    for (uint32_t j : pending) {
      uint32_t r = dst(relays[j]);
      if (in_pass(r, v) && !out_fail(r, d, draw(v, SWIM_STREAM_TRANSIT_PING_OUT, j, 0)) &&
          in_pass(d, r) && !out_fail(d, r, draw(v, SWIM_STREAM_TRANSIT_ACK_OUT, j, 0)) &&
          in_pass(r, d) && !out_fail(r, v, draw(v, SWIM_STREAM_RELAY_ACK_OUT, j, 0))) {
        const uint32_t at = delay_ticks(v, r, v, SWIM_STREAM_PINGREQ_DELAY, j, 0) +
                            delay_ticks(r, d, v, SWIM_STREAM_TRANSIT_PING_DELAY, j, 0) +
                            delay_ticks(d, r, v, SWIM_STREAM_TRANSIT_ACK_DELAY, j, 0) +
                            delay_ticks(r, v, v, SWIM_STREAM_RELAY_ACK_DELAY, j, 0);
        if (at < best) { best = at; first = r; }
      }
    }
    if (late && late - 1 < best) { best = late - 1; first = d; first_gone = late_gone; }
    Member& mv = m[v];
    if (first != NONE && best < relay_ticks && (best > 0 || in_pass(v, first))) {
      if (best == 0) {
        for (size_t i = 0; i < pending.size(); ++i) publish_fd(v, t, first_gone ? SWIM_DEAD : SWIM_ALIVE);
        return;
      }
      mv.relay_due = T + best;  // the first ack arrives then (its inbound filter is applied then)
      mv.relay_ok = true;
      mv.relay_gone = first_gone;
      mv.relay_first = first;
      mv.relay_to = T + relay_ticks;
    } else {
      mv.relay_due = T + relay_ticks;
      mv.relay_ok = false;
    }
    mv.relay_target = t;
    mv.relay_pending = (uint32_t)pending.size();
  }

  bool fd_due(const Member& mv) const {
    return mv.up && (int64_t)T > mv.fd_start && ((int64_t)T - mv.fd_start) % P == 0;
  }
  bool gossip_due(const Member& mv) const {
    return mv.up && (int64_t)T > mv.g_start && ((int64_t)T - mv.g_start) % G == 0;
  }
  bool sync_due(const Member& mv) const {
    return mv.up && mv.sync_on && (int64_t)T > mv.sync_start && ((int64_t)T - mv.sync_start) % S == 0;
  }

  void phase_fd() {
    par(0, n, [&](uint32_t va, uint32_t vb, uint32_t) { phase_fd_range(va, vb); });
  }
  void phase_fd_range(uint32_t va, uint32_t vb) {
    for (uint32_t v = va; v < vb; ++v) {
      Member& mv = m[v];
      if (!mv.up) continue;
      mv.ev_minor = 0;
      if (mv.relay_due == T && mv.relay_ok && !in_pass(v, mv.relay_first)) {
        // the first relayed ack arrives and the inbound filter drops it: no pending relay request
        // completes, they time out (NetworkEmulatorTransport.requestResponse :72-74)
        mv.relay_ok = false;
        mv.relay_due = mv.relay_to;
      }
      if (mv.relay_due == T) {  // relayed acks arrive (:190-199) or the relay timeouts (:200-209)
        uint32_t t = mv.relay_target, k = mv.relay_pending;
        mv.relay_due = 0;
        const uint32_t ok_status = mv.relay_gone ? SWIM_DEAD : SWIM_ALIVE;
        for (uint32_t i = 0; i < k; ++i) publish_fd(v, t, mv.relay_ok ? ok_status : SWIM_SUSPECT);
      }
      if (mv.ack_due == T && mv.ack_ok && !in_pass(v, dst(mv.ack_target))) {
        // the delayed ack arrives and the inbound filter drops it: the ping waits for its timeout
        mv.ack_ok = false;
        mv.ack_due = mv.ack_to;
      }
      if (mv.ack_due == T) {  // the delayed ack arrives, or pingTimeout elapsed (:153-170)
        uint32_t t = mv.ack_target;
        mv.ack_due = 0;
        if (mv.ack_ok) publish_fd(v, t, mv.ack_gone ? SWIM_DEAD : SWIM_ALIVE);
        else ping_req(v, t, mv.ack_late, mv.ack_gone);
      }
      if (fd_due(mv)) {  // doPing (:126-171)
        mv.fd_period++;
        uint32_t t = select_ping_member(v);
        if (t == NONE) continue;
        STT().pings++;
        const uint32_t d = dst(t);  // whoever listens at t's address now
        if (out_fail(v, d, draw(v, SWIM_STREAM_PING_OUT, 0, 0))) {
          ping_req(v, t);  // outbound error -> ping-req right away
        } else {
          // onPing answers DEST_OK, or DEST_GONE from another member at t's address (:227-259) ->
          // computeMemberStatus ALIVE / DEAD (:382-404); the round trip takes both messages' delays
          const bool acked = in_pass(d, v) && !out_fail(d, v, draw(v, SWIM_STREAM_ACK_OUT, 0, 0));
          const uint32_t rtt = acked ? delay_ticks(v, d, v, SWIM_STREAM_PING_DELAY, 0, 0) +
                                           delay_ticks(d, v, v, SWIM_STREAM_ACK_DELAY, 0, 0)
                                     : 0;
          mv.ack_gone = d != t;
          if (acked && rtt == 0 && in_pass(v, d)) {
            publish_fd(v, t, mv.ack_gone ? SWIM_DEAD : SWIM_ALIVE);
          } else {
            // a delayed ack meets the issuer's inbound filter when it arrives (phase above)
            mv.ack_target = t;
            mv.ack_ok = acked && rtt > 0 && rtt < to_ticks;
            mv.ack_due = T + (mv.ack_ok ? rtt : to_ticks);
            mv.ack_to = T + to_ticks;
            mv.ack_late = acked && rtt >= to_ticks ? rtt - to_ticks + 1 : 0;
          }
        }
      }
    }
  }

  // ------------------------------------------------------------------------- phase C: gossip
  // what a GOSSIP_REQ carries that onGossipReq reads (:201-215): the gossip's id and its record — not
  // the sender's GossipState (its infected set stays at the sender; a copy per message would allocate)
  struct GossipRef {
    uint32_t gossiper;
    uint64_t seq;
    Record rec;
  };
  // A delayed GOSSIP_REQ carries its gossip with it (GMsgD, in flight across ticks); a round's
  // messages (GMsg, 20 B: a storm's round materialises 10^8-10^9 of them) refer to the round's table of
  // the gossips its senders sent (ref = table << 26 | index: one table per producer thread, plus one
  // for the delayed messages arriving now)
  struct GMsgD {
    uint32_t to, from, pos;
    GossipRef g;
    uint64_t sent;  // tick of the round that sent it (a delayed message arrives in a later tick)
  };
  struct GMsg {
    uint32_t to, from, pos, ref;
    uint32_t sent;  // (ticks < 2^32)
  };
  static constexpr uint32_t REF_BITS = 26;
  std::map<uint64_t, std::vector<GMsgD>> gossip_in_flight;  // arrival tick -> delayed GOSSIP_REQs

  // selectGossipMembers (GossipProtocolImpl.java:322-343)
  std::vector<uint32_t> select_gossip_members(uint32_t v) {
    Member& mv = m[v];
    const uint32_t F = (uint32_t)cfg.gossip_fanout;
    if (mv.remote.size() < F) return mv.remote;
    if (mv.remote_index < 0 || (uint32_t)mv.remote_index + F > mv.remote.size()) {
      shuffle(v, mv.remote, SWIM_STREAM_GOSSIP_SHUFFLE);
      mv.remote_index = 0;
    }
    std::vector<uint32_t> sel(mv.remote.begin() + mv.remote_index, mv.remote.begin() + mv.remote_index + F);
    mv.remote_index += (int32_t)F;
    return sel;
  }

  void phase_gossip() {
    std::vector<uint32_t> due;
    for (uint32_t v = 0; v < n; ++v)
      if (gossip_due(m[v])) due.push_back(v);
    // GOSSIP_REQs delayed by the network emulator that arrive now (tryDelayOutbound :190-202)
    std::vector<GMsgD> arriving;
    {
      auto it = gossip_in_flight.find(T);
      if (it != gossip_in_flight.end()) {
        arriving.swap(it->second);
        gossip_in_flight.erase(it);
      }
    }
    if (due.empty() && arriving.empty()) return;
    const uint32_t nd = (uint32_t)due.size();
    // C1: period++ and checkGossipSegmentation (:141-146, :217-236)
    par(0, nd, [&](uint32_t a, uint32_t b, uint32_t) {
      for (uint32_t i = a; i < b; ++i) {
        Member& mv = m[due[i]];
        mv.period_used = mv.g_period++;
        for (auto& kv : mv.collectors)
          if (kv.second.size() > (size_t)cfg.gossip_segmentation_threshold) kv.second.clear();
      }
    });
    // C2: spread to selected members, sweep, complete futures (:148-183).  Messages are bucketed by
    // the receiver range of the C3 worker that delivers them ([producer][consumer]).
    const uint32_t nt = std::max(1u, threads);
    std::vector<uint32_t> rb(nt + 1);
    for (uint32_t t = 0; t <= nt; ++t) rb[t] = (uint32_t)((uint64_t)n * t / nt);
    auto consumer = [&](uint32_t to) { return (uint32_t)(std::upper_bound(rb.begin(), rb.end(), to) - rb.begin()) - 1; };
    std::vector<std::vector<std::vector<GMsg>>> bucket(nt, std::vector<std::vector<GMsg>>(nt));
    std::vector<std::vector<GMsgD>> later(nt);  // delayed sends, by producer
    std::vector<std::vector<GossipRef>> sent_tab(nt + 1);  // the gossips sent this round, by producer
    bool any = false;
    par(0, nd, [&](uint32_t a, uint32_t b, uint32_t t) {
      for (uint32_t i = a; i < b; ++i) {
        const uint32_t v = due[i];
        Member& mv = m[v];
        if (mv.gossips.empty()) continue;
        const uint64_t period = mv.period_used;
        std::vector<uint32_t> targets = select_gossip_members(v);
        const int32_t size1 = (int32_t)mv.remote.size() + 1;
        const uint64_t spread = (uint64_t)swim_gossip_periods_to_spread(cfg.gossip_repeat_mult, size1);
        const uint64_t sweep = (uint64_t)swim_gossip_periods_to_sweep(cfg.gossip_repeat_mult, size1);
        // selectGossipsToSend (:311-320): the states in the window, a suffix of the map
        const uint32_t w0 = (uint32_t)mv.window_start(period, spread), nw = (uint32_t)mv.gossips.size();
        const uint32_t tab0 = (uint32_t)sent_tab[t].size();
        for (uint32_t p = w0; p < nw; ++p) {
          const GossipState& g = mv.gossips[p];
          sent_tab[t].push_back(GossipRef{g.gossiper, g.seq, g.rec});
        }
        if (sent_tab[t].size() >= (1u << REF_BITS)) std::abort();  // (refs are 26-bit)
        for (uint32_t j = 0; j < targets.size(); ++j) {
          const uint32_t tg = targets[j], rc = dst(tg);  // sent to tg's address, received by rc
          for (uint32_t p = w0; p < nw; ++p) {
            const GossipState& g = mv.gossips[p];
            if (g.is_infected(tg)) continue;
            STT().gossip_messages++;
            if (out_fail(v, rc, draw(v, SWIM_STREAM_GOSSIP_OUT, j, p))) continue;
            // the receiver's inbound filter applies when the message arrives (listen() :78-83): now,
            // or at the delayed message's arrival tick
            const uint32_t k = delay_ticks(v, rc, v, SWIM_STREAM_GOSSIP_DELAY, j, p);
            if (k) later[t].push_back(GMsgD{rc, v, p, GossipRef{g.gossiper, g.seq, g.rec}, T + k});
            else if (in_pass(rc, v))
              bucket[t][consumer(rc)].push_back(GMsg{rc, v, p, (t << REF_BITS) | (tab0 + p - w0), (uint32_t)T});
          }
        }
        // sweep (:158-164, :350-358)
        mv.sweep_gossips(period, sweep);
        // futures (:167-180, :360-368): the graceful-leave future, and spread() of user gossips — the
        // states before the window (a prefix), looked at only while such a future is pending
        if (mv.leave_pending || mv.user_own) {
          const size_t wf = mv.window_start(period, spread);  // (the states with period > infectionPeriod + spread)
          for (size_t p = 0; p < wf; ++p) {
            GossipState& g = mv.gossips[p];
            if (mv.leave_pending && g.gossiper == mv.leave_gossiper && g.seq == mv.leave_seq) mv.leave_done = true;
            if (g.rec.status == SWIM_GOSSIP_USER && g.gossiper == v) {
              g.rec.status = SWIM_GOSSIP_USER_SPREAD;
              mv.user_own--;
              emit(v, v, SWIM_EV_SPREAD_DONE, SWIM_PHASE_GOSSIP, 0x80000000u | (uint32_t)(g.seq & 0x7fffffffu),
                   g.rec.member);
            }
          }
        }
        // PendingAck waits on LEAVING gossips (onLeavingDetected's spread() Monos): every gossip of one
        // wait has the same infection period, so they complete together — in this round if it finds
        // them disseminated and the sweep above has not dropped them (a swept gossip's Mono never
        // completes)
        for (auto& a : mv.pack)
          if (a.gp && period > a.gp - 1 + spread && !(period > a.gp - 1 + sweep)) {
            a.gp = 0;
            a.ready = std::max(a.ready, T);
          }
      }
    });
    for (auto& lt : later)
      for (auto& x : lt) {
        const uint64_t at = x.sent;
        x.sent = T;
        gossip_in_flight[at].push_back(std::move(x));
      }
    for (auto& x : arriving)  // delayed GOSSIP_REQs arriving now: the receiver's inbound filter now
      if (in_pass(x.to, x.from)) {
        bucket[0][consumer(x.to)].push_back(
            GMsg{x.to, x.from, x.pos, (nt << REF_BITS) | (uint32_t)sent_tab[nt].size(), (uint32_t)x.sent});
        sent_tab[nt].push_back(x.g);
      }
    std::vector<GMsgD>().swap(arriving);
    for (auto& bp : bucket)
      for (auto& bc : bp) any |= !bc.empty();
    if (!any) return;
    // C3: onGossipReq at every receiver, canonical order (sender, slab position) (:201-215)
    par(0, n, [&](uint32_t ra, uint32_t rbnd, uint32_t) {
      std::vector<GMsg> msgs;
      for (uint32_t d = 0; d < nt; ++d)
        if (rb[d] >= ra && rb[d + 1] <= rbnd)
          for (uint32_t pr = 0; pr < nt; ++pr) {
            msgs.insert(msgs.end(), bucket[pr][d].begin(), bucket[pr][d].end());
            std::vector<GMsg>().swap(bucket[pr][d]);  // (this worker is its only reader)
          }
      // canonical order: (receiver, sending round, sender, slab position); keys are unique
      std::sort(msgs.begin(), msgs.end(), [](const GMsg& a, const GMsg& b) {
        if (a.to != b.to) return a.to < b.to;
        if (a.sent != b.sent) return a.sent < b.sent;
        if (a.from != b.from) return a.from < b.from;
        return a.pos < b.pos;
      });
      uint32_t cur = NONE;
      std::vector<PendingAlive> pending;
      for (auto& msg : msgs) {
        const uint32_t r = msg.to;
        Member& mr = m[r];
        if (r != cur) {
          cur = r;
          mr.ev_minor = 0;
          mr.fetch_ctr = 0;
        }
        if (!mr.up) continue;
        const GossipRef& g = sent_tab[msg.ref >> REF_BITS][msg.ref & ((1u << REF_BITS) - 1)];
        if (!mr.collectors[g.gossiper].add((int64_t)g.seq)) continue;
        STT().gossip_accepted++;
        GossipState* state = mr.find_gossip(g.gossiper, g.seq);  // gossips.get(gossipId) (:206)
        if (state == nullptr) {
          GossipState ns;
          ns.gossiper = g.gossiper;
          ns.seq = (uint32_t)g.seq;
          ns.rec = g.rec;
          ns.infection_period = (uint32_t)mr.g_period;
          ns.infected.push_back(msg.from);
          mr.add_gossip(ns);
          if (g.rec.status >= SWIM_GOSSIP_USER) {  // sink.next(gossip.message()) (:209): listen()
            emit(r, g.gossiper, SWIM_EV_GOSSIP, SWIM_PHASE_GOSSIP, next_minor(r), g.rec.member);
            continue;
          }
          // onMembershipGossip (:452-459)
          update_membership(r, g.rec, MEMBERSHIP_GOSSIP, SWIM_PHASE_GOSSIP, pending);
          flush_pending(r, pending, MEMBERSHIP_GOSSIP, SWIM_PHASE_GOSSIP);
        } else {
          state->add_infected(msg.from);
        }
      }
    });
  }

  // ------------------------------------------------------------------------- phase D: SYNC
  // member v's MembershipConfig.seedMembers (:120-130, cleanUpSeedMembers :171-190): its own list
  // (swim_set_member_seeds) or the engine-wide one
  const std::vector<uint32_t>& seeds_of(uint32_t v) const { return m[v].own_seeds ? m[v].seeds : seeds; }
  bool is_seed_of(uint32_t v, uint32_t x) const {
    if (!m[v].own_seeds) return is_seed[x] != 0;
    return std::find(m[v].seeds.begin(), m[v].seeds.end(), x) != m[v].seeds.end();
  }

  // selectSyncAddress (:461-472): uniform over seeds U otherMembers, by seeded rejection sampling.
  uint32_t select_sync_address(uint32_t v) {
    const Member& mv = m[v];
    // seed addresses exclude the local one (cleanUpSeedMembers :171-190)
    uint32_t count = mv.members_size - 1;
    for (uint32_t s : seeds_of(v))
      if (s != v && dst(s) != v && !c_has(mv.row[s], B_IN_MEMBERS)) count++;
    if (count == 0) return NONE;
    auto in_set = [&](uint32_t x) {
      return x != v && (c_has(mv.row[x], B_IN_MEMBERS) || (is_seed_of(v, x) && dst(x) != v));
    };
    for (uint32_t i = 0; i < SWIM_SYNC_SELECT_ATTEMPTS; ++i) {
      uint32_t x = next_int(draw(v, SWIM_STREAM_SYNC_SELECT, 0, i), n);
      if (in_set(x)) return x;
    }
    uint32_t k = next_int(draw(v, SWIM_STREAM_SYNC_SELECT, 1, 0), count);
    for (uint32_t x = 0; x < n; ++x)
      if (in_set(x) && k-- == 0) return x;
    return NONE;
  }

  // syncMembership (:491-509): records in ascending subject order; fetch completions afterwards.
  void sync_membership(uint32_t v, const std::vector<uint64_t>& content, Reason reason, uint32_t phase) {
    std::vector<PendingAlive> pending;
    for (uint32_t x = 0; x < n; ++x) {
      uint64_t c = content[x];
      if (!c_has(c, B_IN_TABLE)) continue;
      STT().sync_records++;
      update_membership(v, Record{x, c_status(c), c_inc(c)}, reason, phase, pending);
    }
    flush_pending(v, pending, reason, phase);
  }

  // SYNCs / SYNC_ACKs the network emulator delays (tryDelayOutbound :190-202 on doSync's send
  // :339-357, onSync's SYNC_ACK send :394-415 and start0's requestResponse :268-276): arrival tick ->
  // messages, each with its content as prepared (the sender's table when it was sent)
  struct SyncFlight {
    uint32_t to, from, ordinal;  // ordinal: the sender's SYNC ordinal, or the SYNC_ACK's inbox rank
    uint64_t sent;
    bool initial, ack;
    std::vector<uint64_t> content;
  };
  std::map<uint64_t, std::vector<SyncFlight>> sync_in_flight;
  // a message merged this tick: arrivals sent in earlier ticks first (canonical order (receiver,
  // sending tick, sender, ordinal / rank))
  // phantom: a deferred SYNC_ACK whose waits completed (PendingAck) — it merges nothing and takes its
  // ack's place at the front of its sender's inbox, in creation order (pre = its seq); wait: the
  // message's Monos are still running, its SYNC_ACK waits (a PendingAck was made)
  struct SyncArr {
    uint32_t to, from, ordinal;
    uint64_t sent;
    bool initial;
    const std::vector<uint64_t>* content;
    uint64_t pre = ~0ull;
    bool phantom = false, wait = false;
  };
  static void sort_arrivals(std::vector<SyncArr>& a) {
    std::stable_sort(a.begin(), a.end(), [](const SyncArr& x, const SyncArr& y) {
      if (x.to != y.to) return x.to < y.to;
      if (x.pre != y.pre) return x.pre < y.pre;
      if (x.sent != y.sent) return x.sent < y.sent;
      if (x.from != y.from) return x.from < y.from;
      return x.ordinal < y.ordinal;
    });
  }

  void phase_sync() {
    const uint32_t nt = std::max(1u, threads);
    std::vector<std::vector<SyncReq>> rq(nt);
    std::vector<std::vector<SyncArr>> ph(nt);
    par(0, n, [&](uint32_t a, uint32_t b, uint32_t t) {
      for (uint32_t v = a; v < b; ++v) {
        Member& mv = m[v];
        if (!mv.up) {  // (a stopped member's waits and deferred acks are void)
          mv.fd_sync.clear();
          mv.pack.clear();
          mv.init_pend = 0;
          continue;
        }
        // PendingAcks whose Monos have all completed: a deferred SYNC_ACK is sent now (doOnSuccess,
        // :399-413), a start0 group leaves the count its doFinally waits for
        if (!mv.pack.empty()) {
          std::vector<PendingAck> keep;
          for (const PendingAck& pa : mv.pack) {
            if (pa.wn || pa.gp || pa.ready > T) { keep.push_back(pa); continue; }
            if (pa.flags & PA_INIT) { mv.init_pend--; continue; }
            SyncArr x{v, pa.to, 0, T, (pa.flags & PA_INITIAL_ACK) != 0, nullptr};
            x.pre = pa.seq;
            x.phantom = true;
            ph[t].push_back(x);
          }
          mv.pack.swap(keep);
        }
        uint32_t k = 0;
        if (sync_due(mv)) {  // doSync (:339-357)
          uint32_t tg = select_sync_address(v);
          if (tg != NONE) rq[t].push_back(SyncReq{v, dst(tg), k++, false, false, false, false});
        }
        for (uint32_t tg : mv.fd_sync) rq[t].push_back(SyncReq{v, dst(tg), k++, false, false, false, false});
        mv.fd_sync.clear();
        if (mv.join_now) {  // start0 initial sync to every seed (:250-291) but its own address
          for (uint32_t s : seeds_of(v))
            if (s != v && dst(s) != v) rq[t].push_back(SyncReq{v, dst(s), k++, true, false, false, false});
        }
      }
    });
    std::vector<SyncReq> reqs;
    for (auto& x : rq) reqs.insert(reqs.end(), x.begin(), x.end());
    std::vector<SyncFlight> arriving;
    {
      auto it = sync_in_flight.find(T);
      if (it != sync_in_flight.end()) {
        arriving.swap(it->second);
        sync_in_flight.erase(it);
      }
    }
    std::vector<SyncArr> phantoms;
    for (auto& x : ph) phantoms.insert(phantoms.end(), x.begin(), x.end());
    if (reqs.empty() && arriving.empty() && phantoms.empty()) {
      finish_joins();
      return;
    }
    // request content: the sender's table when the SYNC is prepared (:485-489)
    std::vector<uint32_t> senders;
    for (auto& q : reqs) senders.push_back(q.from);
    std::sort(senders.begin(), senders.end());
    senders.erase(std::unique(senders.begin(), senders.end()), senders.end());
    std::vector<std::vector<uint64_t>> rows(senders.size());
    par(0, (uint32_t)senders.size(), [&](uint32_t a, uint32_t b, uint32_t) {
      for (uint32_t i = a; i < b; ++i) rows[i] = m[senders[i]].row;
    });
    auto content_of = [&](uint32_t s) -> const std::vector<uint64_t>& {
      return rows[std::lower_bound(senders.begin(), senders.end(), s) - senders.begin()];
    };
    std::vector<SyncArr> in;
    for (size_t i = 0; i < reqs.size(); ++i) {
      SyncReq& q = reqs[i];
      Member& mf = m[q.from];
      STT().syncs++;
      if (q.initial) mf.init_total++;
      // tryFailOutbound (loss) now; the transport's send after tryDelayOutbound meets the receiver
      // — stopped (an error), or its inbound filter — when the message arrives
      // (NetworkEmulatorTransport.send / requestResponse :49-75)
      const uint32_t k = lost(out_loss(q.from, q.to), draw(q.from, SWIM_STREAM_SYNC_OUT, q.ordinal, 0))
                             ? 0u : delay_ticks(q.from, q.to, q.from, SWIM_STREAM_SYNC_DELAY, q.ordinal, 0);
      if (k == 0 && out_fail(q.from, q.to, draw(q.from, SWIM_STREAM_SYNC_OUT, q.ordinal, 0))) {
        q.outfail = true;
        if (q.initial) mf.init_done++;  // an error resumes empty: that source completes now
        continue;
      }
      if (k) {
        sync_in_flight[T + k].push_back(SyncFlight{q.to, q.from, q.ordinal, T, q.initial, false, content_of(q.from)});
        continue;
      }
      if (!in_pass(q.to, q.from)) continue;
      q.delivered = true;
      in.push_back(SyncArr{q.to, q.from, q.ordinal, T, q.initial, &content_of(q.from)});
    }
    std::vector<SyncFlight*> ack_arriving;
    for (auto& f : arriving) {
      if (f.ack) { ack_arriving.push_back(&f); continue; }
      if (!m[f.to].up) {  // the receiver stopped: the transport's send fails now
        if (f.initial && m[f.from].up) m[f.from].init_done++;  // that start0 source completes (an error)
        continue;
      }
      if (!in_pass(f.to, f.from)) continue;  // dropped by the receiver's inbound filter on arrival
      in.push_back(SyncArr{f.to, f.from, f.ordinal, f.sent, f.initial, &f.content});
    }
    in.insert(in.end(), phantoms.begin(), phantoms.end());
    sort_arrivals(in);
    // receivers' inboxes: in[gs[g] .. gs[g + 1])
    std::vector<size_t> gs;
    for (size_t i = 0; i < in.size(); ++i)
      if (i == 0 || in[i].to != in[i - 1].to) gs.push_back(i);
    const uint32_t ng = (uint32_t)gs.size();
    gs.push_back(in.size());
    // D1: onSync at each receiver (:394-415)
    par(0, ng, [&](uint32_t a, uint32_t b, uint32_t) {
      for (uint32_t g = a; g < b; ++g) {
        const uint32_t r = in[gs[g]].to;
        m[r].ev_minor = 0;
        m[r].fetch_ctr = 0;
        for (size_t i = gs[g]; i < gs[g + 1]; ++i) {
          if (in[i].phantom) continue;
          wait_begin(r);
          sync_membership(r, *in[i].content, SYNC, SWIM_PHASE_SYNC);
          in[i].wait = wait_end(r, in[i].from, in[i].initial ? (uint32_t)PA_INITIAL_ACK : 0u);
        }
      }
    });
    // SYNC_ACK content: the receiver's table once all its requests are merged
    std::vector<std::vector<uint64_t>> arows(ng);
    par(0, ng, [&](uint32_t a, uint32_t b, uint32_t) {
      for (uint32_t g = a; g < b; ++g) arows[g] = m[in[gs[g]].to].row;
    });
    std::vector<SyncArr> acks;
    for (uint32_t g = 0; g < ng; ++g) {
      for (size_t i = gs[g]; i < gs[g + 1]; ++i) {
        const SyncArr& q = in[i];
        const uint32_t qr = (uint32_t)(i - gs[g]);
        if (q.wait) continue;  // sent when the message's Monos have completed (a phantom then)
        if (lost(out_loss(q.to, q.from), draw(q.to, SWIM_STREAM_SYNCACK_OUT, qr, 0))) continue;
        const uint32_t k = delay_ticks(q.to, q.from, q.to, SWIM_STREAM_SYNCACK_DELAY, qr, 0);
        if (k) {  // the receiver's state and inbound filter when it arrives
          sync_in_flight[T + k].push_back(SyncFlight{q.from, q.to, qr, T, q.initial, true, arows[g]});
          continue;
        }
        if (!m[q.from].up || !in_pass(q.from, q.to)) continue;
        acks.push_back(SyncArr{q.from, q.to, qr, T, q.initial, &arows[g]});
      }
    }
    for (SyncFlight* f : ack_arriving)
      if (m[f->to].up && in_pass(f->to, f->from))
        acks.push_back(SyncArr{f->to, f->from, f->ordinal, f->sent, f->initial, &f->content});
    sort_arrivals(acks);
    std::vector<size_t> as;
    for (size_t i = 0; i < acks.size(); ++i)
      if (i == 0 || acks[i].to != acks[i - 1].to) as.push_back(i);
    const uint32_t na = (uint32_t)as.size();
    as.push_back(acks.size());
    // D2: SYNC_ACK merge at the original sender (:363-391), INITIAL_SYNC for start0's requests; an
    // initial answer after start0's Flux completed or timed out has no subscriber any more
    par(0, na, [&](uint32_t a, uint32_t b, uint32_t) {
      for (uint32_t g = a; g < b; ++g) {
        const uint32_t s = acks[as[g]].to;
        Member& ms = m[s];
        ms.ev_minor = 0;
        ms.fetch_ctr = 0;
        for (size_t i = as[g]; i < as[g + 1]; ++i) {
          if (acks[i].initial && !ms.init_wait) continue;
          STT().sync_acks++;
          // start0's flatMap (:283): its doFinally waits for the initial merge's Monos too
          if (acks[i].initial) wait_begin(s);
          sync_membership(s, *acks[i].content, acks[i].initial ? INITIAL_SYNC : SYNC, SWIM_PHASE_SYNCACK);
          if (acks[i].initial) wait_end(s, NONE, PA_INIT);
          if (acks[i].initial) {
            ms.init_done++;
            ms.init_last = T;
          }
        }
      }
    });
    finish_joins();
  }

  // start0's doFinally (:285-289).  When every initial SYNC was answered or failed fast, Flux.take
  // completes and doFinally runs once the flatMap's inner Monos — the initial merges' fetches and
  // LEAVING spreads (PendingAck groups, PA_INIT) — have completed: periodic sync starts at the tick the
  // last of them ends.  Otherwise Flux.timeout (:281, restarted at every answer) fires at tick init_last
  // + syncTimeout (an answer arriving in that tick is too late), cancels the inner Monos still running
  // (their fetches complete into nothing) and doFinally runs then.
  void finish_joins() {
    for (uint32_t v = 0; v < n; ++v) {
      Member& mv = m[v];
      mv.join_now = false;
      if (!mv.init_wait) continue;
      int64_t start;
      if (mv.init_done == mv.init_total) {
        if (mv.init_pend) continue;
        start = (int64_t)T;
      } else if (T + 1 >= mv.init_last + sync_to_ticks) {
        start = (int64_t)(mv.init_last + sync_to_ticks);
        std::vector<PendingAck> keep;
        for (const PendingAck& pa : mv.pack)
          if (!(pa.flags & PA_INIT)) keep.push_back(pa);
        mv.pack.swap(keep);
        mv.init_pend = 0;
      } else {
        continue;
      }
      mv.sync_on = true;
      mv.sync_start = start;
      mv.init_wait = false;
    }
  }

  // ------------------------------------------------------------------------- tick
  void start_joins() {
    for (uint32_t v = 0; v < n; ++v) {
      Member& mv = m[v];
      if (!mv.join_pending) continue;
      mv.join_pending = false;
      if (mv.join_addr != NONE) bind_address(v, mv.join_addr);  // the new transport binds the address
      mv.join_addr = NONE;
      mv.up = true;
      mv.joined = true;
      mv.join_now = true;
      mv.init_total = mv.init_done = 0;
      mv.init_last = T;
      mv.init_wait = true;
      mv.pack.clear();
      mv.init_pend = 0;
      mv.fd_start = (int64_t)T;
      mv.g_start = (int64_t)T;
      mv.row[v] = B_IN_TABLE | B_IN_MEMBERS;  // ALIVE inc 0 (MembershipProtocolImpl :146-149)
      mv.table_size = 1;
      mv.members_size = 1;
    }
  }

  // ------------------------------------------------------------------------- FETCH phase
  // delayed GET_METADATA legs arriving this tick, per viewer in issue order; a completed round trip
  // is the fetch's doOnSuccess (apply_alive).  A stopped viewer's round trips are void.
  void phase_fetch() {
    for (uint32_t v = 0; v < n; ++v) {
      Member& mv = m[v];
      if (mv.fq.empty()) continue;
      if (!mv.up) {
        mv.fq.clear();
        continue;
      }
      mv.ev_minor = 0;
      std::vector<PendingFetch> keep;
      for (PendingFetch p : mv.fq) {
        if (p.due > T) {
          keep.push_back(p);
          continue;
        }
        const int r = p.stage == 1 ? fetch_stage1(v, p) : (fetch_stage2(v, p) ? 1 : 0);
        if (r == 2) {
          keep.push_back(p);
          continue;
        }
        if (p.link != NONE) {  // the Mono waiting on it ends now (a response) or at the timeout
          PendingAck* pa = pack_find(v, p.link);
          if (!pa) continue;  // cancelled with start0's Flux: its doOnSuccess never runs
          pa->wn--;
          pa->ready = std::max(pa->ready, r == 1 ? T : p.t0 + mt_ticks);
        }
        if (r == 1) {
          STT().fetch_ok++;
          apply_alive(v, Record{p.s, SWIM_ALIVE, p.inc}, (Reason)p.reason, SWIM_PHASE_FETCH, p.ver);
        }
      }
      mv.fq.swap(keep);
    }
  }

  void step_tick() {
    T += 1;
    st.ticks++;
    start_joins();
    phase_fetch();
    phase_timers();
    phase_fd();
    phase_gossip();
    phase_sync();
    for (uint32_t v = 0; v < n; ++v) {  // graceful leave completes: dispose + transport.stop
      if (m[v].leave_done) {
        m[v].leave_done = false;
        m[v].leave_pending = false;
        m[v].up = false;
      }
    }
  }
};

// =============================================================================== C ABI
extern "C" {

int32_t swim_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  if (!ctr || !key || !out) return SWIM_EINVAL;
  philox4x32_10(ctr, key, out);
  return SWIM_OK;
}

int32_t swim_profile_enable(swim_engine* e, int32_t) { return e ? SWIM_OK : SWIM_EINVAL; }
// the GPU engine's quiet-window fast path has no counterpart here: the oracle runs every tick
int32_t swim_set_quiet_path(swim_engine* e, int32_t) { return e ? SWIM_OK : SWIM_EINVAL; }
int32_t swim_profile_quiet(swim_engine* e, swim_kernel_profile* out) { return swim_profile_merge(e, out); }
int32_t swim_debug_counters(uint64_t* out, uint32_t n, int32_t) {
  if (!out || n > 64) return SWIM_EINVAL;
  std::memset(out, 0, 8ull * n);
  return SWIM_OK;
}
int32_t swim_get_quiet_stats(const swim_engine* e, swim_quiet_stats* out) {
  if (!e || !out) return SWIM_EINVAL;
  std::memset(out, 0, sizeof(*out));
  return SWIM_OK;
}

int32_t swim_profile_merge(swim_engine* e, swim_kernel_profile* out) {
  if (!e || !out) return SWIM_EINVAL;
  std::memset(out, 0, sizeof(*out));
  return SWIM_OK;
}

int32_t swim_profile_fanout(swim_engine* e, swim_kernel_profile* out) { return swim_profile_merge(e, out); }
int32_t swim_profile_deliver(swim_engine* e, swim_kernel_profile* out) { return swim_profile_merge(e, out); }

int32_t swim_kat_overrides(const int32_t* cases, uint32_t n, uint8_t* out) {
  if (n && (!cases || !out)) return SWIM_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    const int32_t* k = cases + 5 * i;
    Record r1{0, (uint32_t)k[0], k[1]};
    Record r0{0, (uint32_t)k[3], k[4]};
    out[i] = is_overrides(r1, k[2] ? &r0 : nullptr) ? 1 : 0;
  }
  return SWIM_OK;
}

int32_t swim_kat_collector(const uint8_t* kinds, const int64_t* values, uint32_t n, int64_t* results) {
  if (n && (!kinds || !values || !results)) return SWIM_EINVAL;
  SeqCollector c;
  for (uint32_t i = 0; i < n; ++i) {
    switch (kinds[i]) {
      case 0: results[i] = c.add(values[i]) ? 1 : 0; break;
      case 1: results[i] = c.contains(values[i]) ? 1 : 0; break;
      case 2: results[i] = (int64_t)c.size(); break;
      case 3: c.clear(); results[i] = 0; break;
      default: return SWIM_EINVAL;
    }
  }
  return SWIM_OK;
}

int32_t swim_ceil_log2(int32_t num) {  // ClusterMath.java:133-135 (32 - numberOfLeadingZeros)
  uint32_t u = (uint32_t)num;
  int32_t nlz = 32;
  while (u) { u >>= 1; nlz--; }
  return 32 - nlz;
}
int32_t swim_gossip_periods_to_spread(int32_t repeat_mult, int32_t cluster_size) {
  return repeat_mult * swim_ceil_log2(cluster_size);
}
int32_t swim_gossip_periods_to_sweep(int32_t repeat_mult, int32_t cluster_size) {
  return 2 * (swim_gossip_periods_to_spread(repeat_mult, cluster_size) + 1);
}
int64_t swim_suspicion_timeout(int32_t suspicion_mult, int32_t cluster_size, int64_t ping_interval) {
  return (int64_t)(suspicion_mult * swim_ceil_log2(cluster_size)) * ping_interval;
}

int32_t swim_config_default(swim_config* c, int32_t preset) {
  if (!c) return SWIM_EINVAL;
  std::memset(c, 0, sizeof(*c));
  c->ping_interval = 1000;
  c->ping_timeout = 500;
  c->ping_req_members = 3;
  c->gossip_interval = 200;
  c->gossip_fanout = 3;
  c->gossip_repeat_mult = 3;
  c->gossip_segmentation_threshold = 1000;
  c->sync_interval = 30000;
  c->sync_timeout = 3000;
  c->suspicion_mult = 5;
  c->removed_members_history_size = 42;
  c->metadata_timeout = 3000;
  c->sync_stagger = 1;
  if (preset == 1) {  // WAN
    c->ping_timeout = 3000;
    c->ping_interval = 5000;
    c->gossip_fanout = 4;
    c->suspicion_mult = 6;
    c->sync_interval = 60000;
    c->metadata_timeout = 10000;
  } else if (preset == 2) {  // Local
    c->ping_timeout = 200;
    c->ping_interval = 1000;
    c->ping_req_members = 1;
    c->gossip_repeat_mult = 2;
    c->gossip_interval = 100;
    c->suspicion_mult = 3;
    c->sync_interval = 15000;
    c->metadata_timeout = 1000;
  } else if (preset != 0) {
    return SWIM_EINVAL;
  }
  return SWIM_OK;
}

static uint32_t gcd_u(uint32_t a, uint32_t b) {
  while (b) { uint32_t t = a % b; a = b; b = t; }
  return a;
}

int32_t swim_create(const swim_config* cfg, uint32_t capacity, uint32_t n_initial, uint64_t seed,
                    swim_engine** out) {
  if (!cfg || !out || capacity == 0 || n_initial > capacity || capacity > (1u << 24)) return SWIM_EINVAL;
  const swim_config& c = *cfg;
  if (c.ping_interval <= 0 || c.ping_timeout <= 0 || c.ping_timeout >= c.ping_interval ||
      c.gossip_interval <= 0 || c.sync_interval <= 0 || c.sync_timeout <= 0 || c.metadata_timeout <= 0 ||
      c.suspicion_mult <= 0 || c.gossip_fanout <= 0 || c.gossip_fanout > 16 || c.ping_req_members > 16 ||
      c.gossip_repeat_mult <= 0)
    return SWIM_EINVAL;
  uint32_t tick = (uint32_t)c.tick_ms;
  if (tick == 0) {
    tick = gcd_u((uint32_t)c.ping_interval, (uint32_t)c.ping_timeout);
    tick = gcd_u(tick, (uint32_t)c.gossip_interval);
    tick = gcd_u(tick, (uint32_t)c.sync_interval);
    tick = gcd_u(tick, (uint32_t)c.sync_timeout);
  }
  if (c.ping_interval % tick || c.ping_timeout % tick || c.gossip_interval % tick || c.sync_interval % tick ||
      c.sync_timeout % tick)
    return SWIM_EINVAL;
  swim_engine* e = new (std::nothrow) swim_engine();
  if (!e) return SWIM_ENOMEM;
  e->cfg = c;
  e->n = capacity;
  e->seed = seed;
  e->key[0] = (uint32_t)seed;
  e->key[1] = (uint32_t)(seed >> 32);
  e->tick_ms = tick;
  e->P = (uint32_t)c.ping_interval / tick;
  e->to_ticks = (uint32_t)c.ping_timeout / tick;
  e->relay_ticks = e->P - e->to_ticks;
  e->G = (uint32_t)c.gossip_interval / tick;
  e->S = (uint32_t)c.sync_interval / tick;
  e->sync_to_ticks = (uint32_t)c.sync_timeout / tick;
  e->mt_ticks = (uint32_t)(((int64_t)c.metadata_timeout + tick - 1) / tick);
  try {
    e->m.resize(capacity);
    e->is_seed.assign(capacity, 0);
    e->default_loss.assign(capacity, 0);
    e->default_delay.assign(capacity, 0);
    e->meta_ver.assign(capacity, 0);
    e->default_inbound.assign(capacity, 1);
    e->group.assign(capacity, 0);
    for (auto& mm : e->m) mm.row.assign(capacity, 0);
  } catch (...) {
    delete e;
    return SWIM_ENOMEM;
  }
  // Converged initial cluster.  Initialisation may use threads; ticks never do.
  const uint64_t conv = B_IN_TABLE | B_IN_MEMBERS | B_ALIVE_EMITTED | B_HAS_METADATA;
  auto init_range = [&](uint32_t lo, uint32_t hi) {
    for (uint32_t v = lo; v < hi; ++v) {
      Member& mv = e->m[v];
      mv.up = mv.joined = true;
      for (uint32_t s = 0; s < n_initial; ++s) mv.row[s] = conv;
      mv.row[v] = B_IN_TABLE | B_IN_MEMBERS;  // self: ALIVE inc 0
      mv.table_size = n_initial;
      mv.members_size = n_initial;
      mv.ping_members.reserve(n_initial ? n_initial - 1 : 0);
      for (uint32_t s = 0; s < n_initial; ++s)
        if (s != v) mv.ping_members.push_back(s);
      mv.remote = mv.ping_members;
      for (uint32_t i = (uint32_t)mv.ping_members.size(); i > 1; --i) {
        uint32_t j = next_int(e->draw(v, SWIM_STREAM_INIT_PING, 0, i, 0), i);
        std::swap(mv.ping_members[i - 1], mv.ping_members[j]);
      }
      for (uint32_t i = (uint32_t)mv.remote.size(); i > 1; --i) {
        uint32_t j = next_int(e->draw(v, SWIM_STREAM_INIT_REMOTE, 0, i, 0), i);
        std::swap(mv.remote[i - 1], mv.remote[j]);
      }
      mv.remote_index = 0;
      mv.sync_on = true;
      mv.sync_start = c.sync_stagger ? -(int64_t)next_int(e->draw(v, SWIM_STREAM_INIT_SYNC_PHASE, 0, 0, 0), e->S) : 0;
      if (c.timer_stagger) {  // members of a real cluster start at different instants
        mv.fd_start = -(int64_t)next_int(e->draw(v, SWIM_STREAM_INIT_FD_PHASE, 0, 0, 0), e->P);
        mv.g_start = -(int64_t)next_int(e->draw(v, SWIM_STREAM_INIT_GOSSIP_PHASE, 0, 0, 0), e->G);
      }
    }
  };
  unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n_initial < 4096) hw = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < hw; ++t) {
    uint32_t lo = (uint32_t)((uint64_t)n_initial * t / hw), hi = (uint32_t)((uint64_t)n_initial * (t + 1) / hw);
    if (hw == 1) init_range(lo, hi); else th.emplace_back(init_range, lo, hi);
  }
  for (auto& x : th) x.join();
  *out = e;
  return SWIM_OK;
}

// Oracle only (not in swim.h): worker threads of the per-member phase loops (the CPU baseline's
// all-core leg; results are identical for every thread count).  0 = hardware concurrency.
int32_t swim_oracle_set_threads(swim_engine* e, int32_t threads) {
  if (!e || threads < 0) return SWIM_EINVAL;
  e->threads = threads ? (uint32_t)threads : std::max(1u, std::thread::hardware_concurrency());
  return SWIM_OK;
}

int32_t swim_destroy(swim_engine* e) {
  delete e;
  return SWIM_OK;
}

// Row sharding is a deployment of the same lockstep semantics: a sharded GPU run
// must equal the unsharded one bit for bit.  The oracle is the unsharded restatement, so it only
// accepts world = 1 and answers for the whole cluster.
int32_t swim_comm_unique_id(uint8_t* out) {
  if (!out) return SWIM_EINVAL;
  std::memset(out, 0, SWIM_COMM_ID_BYTES);
  return SWIM_OK;
}

int32_t swim_create_shard(const swim_config* cfg, uint32_t capacity, uint32_t n_initial, uint64_t seed, int32_t rank,
                          int32_t world, const uint8_t*, swim_engine** out) {
  if (world != 1 || rank != 0) return SWIM_EINVAL;
  return swim_create(cfg, capacity, n_initial, seed, out);
}

int32_t swim_exchange_info(const swim_engine* e, uint32_t* flags) {  // (the oracle never exchanges)
  if (!e || !flags) return SWIM_EINVAL;
  *flags = 0;
  return SWIM_OK;
}

int32_t swim_shard_info(const swim_engine* e, int32_t* rank, int32_t* world, uint32_t* lo, uint32_t* count) {
  if (!e) return SWIM_EINVAL;
  if (rank) *rank = 0;
  if (world) *world = 1;
  if (lo) *lo = 0;
  if (count) *count = e->n;
  return SWIM_OK;
}

int32_t swim_step_ticks(swim_engine* e, uint32_t ticks) {
  if (!e) return SWIM_EINVAL;
  for (uint32_t i = 0; i < ticks; ++i) e->step_tick();
  return SWIM_OK;
}

int32_t swim_step(swim_engine* e, uint32_t periods) {
  if (!e) return SWIM_EINVAL;
  return swim_step_ticks(e, periods * e->P);
}

int32_t swim_now(const swim_engine* e, uint64_t* tick, uint32_t* tick_ms, uint32_t* tpp) {
  if (!e) return SWIM_EINVAL;
  if (tick) *tick = e->T;
  if (tick_ms) *tick_ms = e->tick_ms;
  if (tpp) *tpp = e->P;
  return SWIM_OK;
}

int32_t swim_set_member_seeds(swim_engine* e, uint32_t v, const uint32_t* seeds, uint32_t n_seeds) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  Member& mv = e->m[v];
  if (!seeds && n_seeds == 0xffffffffu) {  // back on the engine-wide list
    mv.own_seeds = false;
    mv.seeds.clear();
    return SWIM_OK;
  }
  if (n_seeds && !seeds) return SWIM_EINVAL;
  std::vector<uint32_t> s;
  for (uint32_t i = 0; i < n_seeds; ++i) {
    if (seeds[i] >= e->n) return SWIM_EINVAL;
    if (std::find(s.begin(), s.end(), seeds[i]) == s.end()) s.push_back(seeds[i]);  // LinkedHashSet
  }
  mv.seeds = std::move(s);
  mv.own_seeds = true;
  return SWIM_OK;
}

int32_t swim_set_seeds(swim_engine* e, const uint32_t* seeds, uint32_t n_seeds) {
  if (!e || (n_seeds && !seeds)) return SWIM_EINVAL;
  std::vector<uint32_t> s;
  for (uint32_t i = 0; i < n_seeds; ++i) {
    if (seeds[i] >= e->n) return SWIM_EINVAL;
    if (std::find(s.begin(), s.end(), seeds[i]) == s.end()) s.push_back(seeds[i]);  // LinkedHashSet
  }
  e->seeds = s;
  std::fill(e->is_seed.begin(), e->is_seed.end(), 0);
  for (uint32_t x : s) e->is_seed[x] = 1;
  return SWIM_OK;
}

int32_t swim_kill(swim_engine* e, uint32_t mm) {
  if (!e || mm >= e->n) return SWIM_EINVAL;
  if (!e->m[mm].up) return SWIM_ESTATE;
  e->m[mm].up = false;
  e->m[mm].leave_pending = false;
  return SWIM_OK;
}

int32_t swim_leave(swim_engine* e, uint32_t v, int32_t stop_after) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  Member& mv = e->m[v];
  if (!mv.up) return SWIM_ESTATE;
  // leaveCluster (:233-242)
  uint64_t& c = mv.row[v];
  Record r{v, SWIM_LEAVING, c_inc(c) + 1};
  c = c_with_record(c, r.status, r.inc);
  e->spread_gossip(v, r, SWIM_ORIG_LEAVE);
  if (stop_after) {
    mv.leave_pending = true;
    mv.leave_gossiper = v;
    mv.leave_seq = mv.g_counter - 1;
  }
  return SWIM_OK;
}

// external SYNC ingestion (swim.h): onSyncAck (MembershipProtocolImpl.java:363-391) between ticks
int32_t swim_ingest_sync(swim_engine* e, uint32_t v, const swim_record* records, uint32_t n, int32_t initial) {
  if (!e || v >= e->n || n > e->n || (n && !records)) return SWIM_EINVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (records[i].member >= e->n || records[i].status >= SWIM_DEAD || records[i].inc < 0) return SWIM_EINVAL;
  if (!e->m[v].up) return SWIM_ESTATE;
  const Reason reason = initial ? INITIAL_SYNC : SYNC;
  // the control phase's event minors and fetch draws run on across the operations of one tick (two
  // ingestions between the same ticks: distinct event keys, distinct draws)
  if (e->m[v].ctl_tick1 != e->T + 1) {
    e->m[v].ev_minor = 0;
    e->m[v].fetch_ctr = 0;
    e->m[v].ctl_tick1 = e->T + 1;
  }
  std::vector<PendingAlive> pending;
  for (uint32_t i = 0; i < n; ++i)
    e->update_membership(v, Record{records[i].member, records[i].status, records[i].inc}, reason, SWIM_PHASE_CONTROL,
                         pending);
  e->flush_pending(v, pending, reason, SWIM_PHASE_CONTROL);
  e->STT().sync_acks++;
  e->STT().sync_records += n;
  return SWIM_OK;
}

int32_t swim_spread(swim_engine* e, uint32_t v, uint32_t payload) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  if (!e->m[v].up) return SWIM_ESTATE;
  e->spread_user(v, payload);  // GossipProtocolImpl.spread (:126-130)
  return SWIM_OK;
}

int32_t swim_join(swim_engine* e, uint32_t v) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  Member& mv = e->m[v];
  if (mv.joined || mv.up || mv.join_pending) return SWIM_ESTATE;
  mv.join_pending = true;
  return SWIM_OK;
}

int32_t swim_join_at(swim_engine* e, uint32_t v, uint32_t addr_of) {
  if (!e || v >= e->n || addr_of >= e->n || addr_of == v) return SWIM_EINVAL;
  const uint32_t holder = e->dst(addr_of);
  if (e->m[holder].up || e->m[holder].join_pending) return SWIM_ESTATE;  // the address is in use
  for (uint32_t x = 0; x < e->n; ++x)
    if (x != v && e->m[x].join_pending && e->m[x].join_addr != NONE && e->dst(e->m[x].join_addr) == holder)
      return SWIM_ESTATE;
  if (int32_t rc = swim_join(e, v)) return rc;
  e->m[v].join_addr = addr_of;
  return SWIM_OK;
}

int32_t swim_set_default_loss(swim_engine* e, uint32_t mm, int32_t pct) {
  if (!e || pct < 0 || pct > 100) return SWIM_EINVAL;
  if (mm == 0xffffffffu) { std::fill(e->default_loss.begin(), e->default_loss.end(), pct); return SWIM_OK; }
  if (mm >= e->n) return SWIM_EINVAL;
  e->default_loss[mm] = pct;
  return SWIM_OK;
}

int32_t swim_set_link_loss(swim_engine* e, uint32_t src, uint32_t dst, int32_t pct) {
  if (!e || src >= e->n || dst >= e->n || pct > 100) return SWIM_EINVAL;
  if (pct < 0) e->link_loss.erase({src, dst}); else e->link_loss[{src, dst}] = pct;
  return SWIM_OK;
}

int32_t swim_set_namespaces(swim_engine* e, const uint16_t* ns_of_member, uint32_t n_ns, const uint8_t* related) {
  if (!e) return SWIM_EINVAL;
  if (n_ns == 0 || !ns_of_member) {
    e->n_ns = 0;
    return SWIM_OK;
  }
  if (!related || n_ns > 4096) return SWIM_EINVAL;
  for (uint32_t i = 0; i < e->n; ++i)
    if (ns_of_member[i] >= n_ns) return SWIM_EINVAL;
  // the converged start holds every initial member in every initial member's table
  std::vector<uint8_t> used(n_ns, 0);
  for (uint32_t a = 0; a < e->n; ++a)
    if (e->m[a].joined) used[ns_of_member[a]] = 1;
  for (uint32_t x = 0; x < n_ns; ++x)
    for (uint32_t y = 0; y < n_ns; ++y)
      if (used[x] && used[y] && !related[(size_t)x * n_ns + y]) return SWIM_ESTATE;
  e->ns.assign(ns_of_member, ns_of_member + e->n);
  e->ns_rel.assign(related, related + (size_t)n_ns * n_ns);
  e->n_ns = n_ns;
  return SWIM_OK;
}

int32_t swim_update_metadata(swim_engine* e, uint32_t v) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  Member& mv = e->m[v];
  if (!mv.up) return SWIM_ESTATE;
  if (e->meta_seen.empty()) e->meta_seen.assign(e->n, std::vector<uint32_t>(e->n, 0));
  e->meta_ver[v]++;  // metadataStore.updateMetadata(metadata) (ClusterImpl.java:497-500)
  // updateIncarnation (MembershipProtocolImpl.java:214-226): ALIVE inc+1, spread
  uint64_t& c = mv.row[v];
  Record r{v, SWIM_ALIVE, c_inc(c) + 1};
  c = c_with_record(c, r.status, r.inc);
  e->spread_gossip(v, r, SWIM_ORIG_METADATA);
  return SWIM_OK;
}

int32_t swim_set_default_delay(swim_engine* e, uint32_t mm, int32_t mean_ms) {
  if (!e || mean_ms < 0) return SWIM_EINVAL;
  if (mm != 0xffffffffu && mm >= e->n) return SWIM_EINVAL;
  if (mean_ms > 0 && !e->delay_mean_acceptable(mean_ms)) return SWIM_EINVAL;  // swim_delay.h cap, 4,096 tables
  e->ensure_delay_tab(mean_ms);
  if (mm == 0xffffffffu) std::fill(e->default_delay.begin(), e->default_delay.end(), mean_ms);
  else e->default_delay[mm] = mean_ms;
  return SWIM_OK;
}

int32_t swim_set_link_delay(swim_engine* e, uint32_t src, uint32_t dst, int32_t mean_ms) {
  if (!e || src >= e->n || dst >= e->n) return SWIM_EINVAL;
  if (mean_ms < 0) {
    e->link_delay.erase({src, dst});
  } else {
    if (mean_ms > 0 && !e->delay_mean_acceptable(mean_ms)) return SWIM_EINVAL;  // swim_delay.h cap, 4,096 tables
    e->ensure_delay_tab(mean_ms);
    e->link_delay[{src, dst}] = mean_ms;
  }
  return SWIM_OK;
}

int32_t swim_set_link_inbound(swim_engine* e, uint32_t dst, uint32_t src, int32_t pass) {
  if (!e || src >= e->n || dst >= e->n) return SWIM_EINVAL;
  if (pass < 0) e->link_inbound.erase({dst, src}); else e->link_inbound[{dst, src}] = pass ? 1 : 0;
  return SWIM_OK;
}

int32_t swim_set_default_inbound(swim_engine* e, uint32_t mm, int32_t pass) {
  if (!e) return SWIM_EINVAL;
  if (mm == 0xffffffffu) { std::fill(e->default_inbound.begin(), e->default_inbound.end(), pass ? 1 : 0); return SWIM_OK; }
  if (mm >= e->n) return SWIM_EINVAL;
  e->default_inbound[mm] = pass ? 1 : 0;
  return SWIM_OK;
}

int32_t swim_set_partition(swim_engine* e, const uint16_t* g) {
  if (!e) return SWIM_EINVAL;
  if (!g) { e->partition = false; return SWIM_OK; }
  e->partition = true;
  std::memcpy(e->group.data(), g, sizeof(uint16_t) * e->n);
  return SWIM_OK;
}

int32_t swim_read_view(swim_engine* e, uint32_t v, uint64_t* out) {
  if (!e || v >= e->n || !out) return SWIM_EINVAL;
  std::memcpy(out, e->m[v].row.data(), sizeof(uint64_t) * e->n);
  return SWIM_OK;
}

int32_t swim_drain_events(swim_engine* e, swim_event* out, size_t cap, size_t* n_out) {
  if (!e || (cap && !out)) return SWIM_EINVAL;
  std::stable_sort(e->events.begin(), e->events.end(), [](const swim_event& a, const swim_event& b) {
    if (a.tick != b.tick) return a.tick < b.tick;
    if (a.viewer != b.viewer) return a.viewer < b.viewer;
    if (a.phase != b.phase) return a.phase < b.phase;
    return a.minor < b.minor;
  });
  size_t k = std::min(cap, e->events.size());
  if (k) std::memcpy(out, e->events.data(), k * sizeof(swim_event));
  e->events.erase(e->events.begin(), e->events.begin() + (ptrdiff_t)k);
  if (n_out) *n_out = k;
  return SWIM_OK;
}

int32_t swim_get_stats(swim_engine* e, swim_stats* out) {
  if (!e || !out) return SWIM_EINVAL;
  *out = e->st;
  return SWIM_OK;
}

int32_t swim_read_member(swim_engine* e, uint32_t v, swim_member_state* o) {
  if (!e || v >= e->n || !o) return SWIM_EINVAL;
  const Member& mv = e->m[v];
  std::memset(o, 0, sizeof(*o));
  o->up = mv.up;
  o->joined = mv.joined;
  o->leave_pending = mv.leave_pending;
  o->join_pending = mv.join_pending;
  o->remote_idx = mv.remote_index;
  o->fd_period = mv.fd_period;
  o->ping_cursor = mv.ping_index;
  o->ping_len = (uint32_t)mv.ping_members.size();
  o->remote_len = (uint32_t)mv.remote.size();
  o->gossip_len = (uint32_t)mv.gossips.size();
  o->gossip_period = mv.g_period;
  o->gossip_counter = mv.g_counter;
  o->table_size = mv.table_size;
  o->members_size = mv.members_size;
  o->fd_start = mv.fd_start;
  o->gossip_start = mv.g_start;
  o->sync_start = mv.sync_start;
  o->sync_on = mv.sync_on;
  o->ack_target = mv.ack_due ? mv.ack_target : 0xffffffffu;
  o->ack_due = mv.ack_due;
  o->relay_target = mv.relay_due ? mv.relay_target : 0xffffffffu;
  o->relay_pending = mv.relay_due ? mv.relay_pending : 0;
  o->relay_due = mv.relay_due;
  o->leave_gossiper = mv.leave_pending ? mv.leave_gossiper : 0xffffffffu;
  o->leave_seq = mv.leave_pending ? mv.leave_seq : 0;
  o->pending_acks = (uint32_t)mv.pack.size();
  return SWIM_OK;
}

static int32_t copy_list(const std::vector<uint32_t>& l, uint32_t* out, uint32_t cap, uint32_t* len) {
  if (len) *len = (uint32_t)l.size();
  if (out) std::memcpy(out, l.data(), sizeof(uint32_t) * std::min<size_t>(cap, l.size()));
  return SWIM_OK;
}

int32_t swim_read_ping_list(swim_engine* e, uint32_t v, uint32_t* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  return copy_list(e->m[v].ping_members, out, cap, len);
}

int32_t swim_read_remote_list(swim_engine* e, uint32_t v, uint32_t* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  return copy_list(e->m[v].remote, out, cap, len);
}

int32_t swim_read_gossips(swim_engine* e, uint32_t v, swim_gossip* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  const auto& gs = e->m[v].gossips;
  if (len) *len = (uint32_t)gs.size();
  for (uint32_t i = 0; i < gs.size() && i < cap && out; ++i) {
    const GossipState& g = gs[i];
    swim_gossip& o = out[i];
    o.gossiper = g.gossiper;
    o.subject = g.rec.member;
    o.seq = g.seq;
    o.inc = g.rec.inc;
    o.status = g.rec.status;
    o.infection_period = g.infection_period;
    o.infected[0] = g.infected.size() > 0 ? g.infected[0] : 0xffffffffu;
    o.infected[1] = g.infected.size() > 1 ? g.infected[1] : 0xffffffffu;
  }
  return SWIM_OK;
}

int32_t swim_read_collector(swim_engine* e, uint32_t v, uint32_t gossiper, swim_interval* out, uint32_t cap,
                            uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  auto& cols = e->m[v].collectors;
  auto it = cols.find(gossiper);
  if (it == cols.end()) { if (len) *len = 0; return SWIM_OK; }
  if (len) *len = (uint32_t)it->second.iv.size();
  uint32_t i = 0;
  for (auto& kv : it->second.iv) {
    if (i >= cap || !out) break;
    out[i].lo = (uint64_t)kv.first;
    out[i].hi = (uint64_t)kv.second;
    ++i;
  }
  return SWIM_OK;
}

}  // extern "C"
