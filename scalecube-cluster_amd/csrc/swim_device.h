// swim_device.h — device data layout and per-viewer protocol logic of the lockstep SWIM engine.
//
// Layout: everything is structure-of-arrays in HBM, row-major per viewer.
//   recs    u32[N][N]   view record word per (viewer, subject); aux u32[N][N] the side maps
//   ping    u32[N][N]   FailureDetectorImpl.pingMembers of each viewer (ArrayList order)
//   remote  u32[N][N]   GossipProtocolImpl.remoteMembers of each viewer
//   slab    GossipDev[N][gcap]  live GossipStates, insertion order
//   gix     u32[N][2 gcap]      lazily built (gossiper, seq) -> slab serial index (gix_find)
//   coll    CollEnt[N][hcap]    SequenceIdCollector per (viewer, gossiper), open addressing, one
//                               interval inline; more spill to size-tiered interval blocks
//   mem     MemberDev[N]        scalar per-member protocol state
//
// The functions below run on ONE thread that owns viewer v for the duration of a phase (the
// canonical sequential semantics of DESIGN.md §3); parallelism is across viewers, and inside
// SYNC row merges across subjects (swim_kernels.h).  Citations are to
// /root/reference/cluster/src/main/java/io/scalecube/cluster/ unless noted.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/swim.h"
#include "../../include/swim_delay.h"
#include "../../include/swim_rng.h"

namespace swimdev {

constexpr uint32_t NONE = 0xffffffffu;
// Ctx.mflag bits (MF_PACK: the member holds PendingAcks, see PAck)
enum : uint32_t { MF_FDSYNC = 1, MF_JOIN = 2, MF_LEAVE = 4, MF_PACK = 8 };
constexpr int NTIER = 4;       // spilled-collector block tiers
constexpr int FD_SYNC_MAX = 33;  // FD-triggered SYNCs per member per tick (<= 2k+1)

// error bits (stats.capacity_errors / SWIM_ECAPACITY)
enum : uint32_t {
  ERR_SLAB = 1u << 0, ERR_INTERVALS = 1u << 1, ERR_HASH = 1u << 2, ERR_WHEEL = 1u << 3,
  ERR_EVENTS = 1u << 4, ERR_MSGS = 1u << 5, ERR_SNAP = 1u << 6, ERR_INFECTED = 1u << 7,
  ERR_FDSYNC = 1u << 8, ERR_INS = 1u << 9, ERR_REQS = 1u << 10, ERR_PEND = 1u << 11, ERR_INC = 1u << 12,
  ERR_PAGES = 1u << 13,  // the gossip inbox page pool ran dry
  ERR_INBOX = 1u << 14,  // one receiver's gossip inbox outgrew its page table
  ERR_COLL_TOP = 1u << 15,  // a collector outgrew the top spill tier (ERR_INTERVALS: a tier's pool ran dry)
  ERR_DELAY = 1u << 16,     // more delayed GOSSIP_REQs arrive in one tick than a delay bucket holds
  ERR_XPTR = 1u << 17,      // SWIM_DEBUG_SYNC: a sharded tick would dereference a null exchange pointer
  ERR_SDELAY = 1u << 18,    // delayed SYNCs / SYNC_ACKs: a delay bucket or the park slots ran out
  ERR_FETCHQ = 1u << 19,    // more delayed GET_METADATA round trips in flight than the fetch queue holds
  ERR_PACK = 1u << 20,      // a member holds more merged messages waiting on their Monos than pa_cap
};

// A GET_METADATA round trip in flight under message delay (MetadataStoreImpl.fetchMetadata :146-185):
// stage 1 = the request travelling to the subject's address d, stage 2 = the response travelling
// back; due = the arrival tick of the current leg; draws stay keyed by the issue tick t0.  Per viewer
// a chain in issue order (next), in the queue of the tick it was written in (Ctx.fq, by tick parity).
struct FetchEnt {
  uint32_t s;
  int32_t inc;
  uint32_t f;
  uint32_t info;  // phase | reason << 4 | stage << 8
  uint32_t d, ver, t0, due, next;
  uint32_t link;  // seq of the viewer's PAck waiting on this fetch, or NONE
};

// A merged message whose updateMembership Monos have not all completed (syncMembership
// :491-509, Flux.mergeDelayError): onSync's SYNC_ACK waits for them (MembershipProtocolImpl.java
// :394-415, prepared and sent in doOnSuccess), and so does start0's doFinally for an initial SYNC_ACK
// merged through its flatMap (:277-289).  A Mono waits on an ALIVE admission's metadata fetch (ended
// by its response, at once by a failed send, else at metadataTimeout) or on a new LEAVING record's
// gossip (onLeavingDetected returns spreadMembershipGossip: GossipProtocolImpl.spread's Mono ends when
// the gossip most likely disseminated, :167-180).  Per member, in creation order (Ctx.pa, pa_n);
// oracle: PendingAck.
constexpr uint32_t PA_CAP = 64;  // pa_cap's base (grown before join bursts: grow_for_joins)
enum : uint32_t { PA_INITIAL_ACK = 1, PA_INIT = 2 };  // the deferred ack answers start0 / a start0 group
struct PAck {
  uint32_t to;     // the SYNC's sender (PA_INIT: unused)
  uint32_t flags;
  uint32_t wn;     // fetches still in flight
  uint32_t ready;  // the tick the last completed or timed-out wait ended
  uint32_t gp;     // 1 + the infection period of the LEAVING gossips waited on (0: none)
  uint32_t seq;
};

// stats slots (swim_stats order)
enum { ST_TICKS, ST_PINGS, ST_PING_REQS, ST_FD_EVENTS, ST_GOSSIPS_CREATED, ST_GOSSIP_MESSAGES,
       ST_GOSSIP_ACCEPTED, ST_SYNCS, ST_SYNC_ACKS, ST_SYNC_RECORDS, ST_FETCHES, ST_FETCH_OK,
       ST_TIMERS_FIRED, ST_EVENTS, ST_CAPACITY_ERRORS,
       ST_MERGE_MSGS, ST_MERGE_RECORDS,  // (unused slots, kept for the stats layout)
       ST_ORIG0,  // 7 slots: gossips_created by SWIM_ORIG_* reason (swim_stats.gossips_by_reason)
       ST_COUNT = ST_ORIG0 + 7 };
static_assert(ST_COUNT == 24, "stats slots");

enum Reason { R_FD_EVENT, R_GOSSIP, R_SYNC, R_INITIAL_SYNC, R_TIMEOUT };

constexpr uint64_t B_IN_TABLE = 1ull << 34, B_IN_MEMBERS = 1ull << 35, B_ALIVE_EMITTED = 1ull << 36,
                   B_HAS_TIMER = 1ull << 37, B_HAS_METADATA = 1ull << 38;

// Per-member scalar state of an OWNED member (index v - Ctx.lo).  Whether a member's transport
// is up is replicated on every shard (Ctx.up), because every sender reads it.
// The per-member words every gossip tick touches for every member (doSpreadGossip's period++ and
// the live-gossip test), kept out of MemberDev so that a round costs one coalesced 16-B word per
// member instead of two MemberDev cache lines.
struct alignas(16) GossipSched {
  uint32_t next;    // tick of the next gossip round (schedule phase g_start, period G; kept while down)
  uint32_t period;  // GossipProtocolImpl.currentPeriod (< 2^28: ERR_INC)
  uint32_t len;     // live gossips in the member's slab (GossipProtocolImpl.gossips.size())
  uint32_t base;    // the slab is a ring: gossip p (insertion order) lives at (base + p) mod gcap; the
                    // sweep drops a prefix by advancing base (nothing moves)
};

struct alignas(16) MemberDev {
  // first 64 B: every word the quiet scan reads and the quiet apply writes (k_quiet_scan /
  // k_quiet_apply: one 64-B sector per member)
  uint64_t ack_due, relay_due;
  uint32_t ping_cursor, ping_len, table_size, fd_sync_cnt;
  uint32_t ins_rank;  // this phase's deferred pingMembers inserts (op chain: ins_head / ins_tail)
  uint8_t join_now, join_pending, leave_pending;
  uint8_t init_wait;  // start0's initial-sync Flux is still subscribed (init_total / init_done)
  uint64_t fd_period;
  uint32_t ev_minor, fetch_ctr;
  uint64_t g_counter, leave_seq;
  int64_t fd_start, g_start, sync_start;
  uint32_t ack_target, relay_target, relay_pending;
  uint32_t remote_len;
  int32_t remote_idx;
  uint32_t members_size, leave_gossiper;
  uint32_t init_total, init_done;
  uint32_t ins_head, ins_tail;
  uint32_t gix_base, gix_used;  // serial of slab[0]; gix slots taken since the index was (re)built
  uint32_t ack_late;  // 1 + ticks after the ping timeout that a late direct ack arrives (0 = none)
  uint64_t ack_to, relay_to;  // the ping's / the relay requests' timeout tick (an ack the inbound
                              // filter drops on arrival leaves them waiting until then)
  uint32_t relay_first;       // the sender of the first relayed ack (filtered when it arrives)
  uint32_t init_last;  // start0's initial sync: tick of the last answer (or of the start)
  uint32_t user_live;  // this member's own user gossips whose spread() has not completed (the emit
                       // round reads the states past the spreading window only while one is pending)
  uint8_t joined, leave_done, sync_on, gix_valid;
  uint8_t ack_ok;    // ack_due is the tick the (delayed) ack arrives, not the ping timeout
  uint8_t relay_ok;  // relay_due is the tick the first relayed ack arrives, not the timeout
  uint8_t ack_gone, relay_gone;  // that ack says DEST_GONE (another member listens at the target's address)
  // PendingAcks (PAck): the next seq, the start0 groups pending; the waits of the message being merged
  // (w_link1 = 1 + the seq its PAck will take, 0 outside such a merge)
  uint32_t pack_seq, init_pend;
  uint32_t w_link1, w_n, w_ready, w_gp;
  uint32_t ctl_tick1;  // 1 + the tick of the member's last control-phase operation (swim_ingest_sync)
  uint32_t clr_serial;  // slab serial at the member's last collector clear (states below it predate it)
};
static_assert(sizeof(MemberDev) == 224, "MemberDev: 224 B (the quiet scan's words in the first 64-B sector)");

// GossipState + Gossip + MembershipRecord payload, 48 B.  GossipState.infected gains a member only
// when the collector accepts the sequence id (onGossipReq :205-212): the first sender, plus one more
// per re-acceptance after checkGossipSegmentation cleared the collector; GINF entries hold that
// (ERR_INFECTED beyond, never a silent truncation).
constexpr int GINF = 6;
struct GossipDev {
  uint32_t gossiper, subject, seq, inf_period;
  int32_t inc;
  uint32_t status;
  uint32_t inf[GINF];  // GossipState.infected in insertion order (NONE = empty)
};
__device__ __forceinline__ bool gossip_infected(const GossipDev& g, uint32_t m) {
  bool r = false;
#pragma unroll
  for (int k = 0; k < GINF; ++k) r |= g.inf[k] == m;
  return r;
}

// The slab stores a GossipDev in two parts at the same position: 16 hot bytes — all that a gossip
// round reads for every live gossip (window, sweep, futures, first infected member, receipt key) —
// and 8 cold bytes (the payload record) read only for the gossips a round actually sends or moves:
// 24 B per GossipState.  GossipState.infected beyond its first member (`more`: only after a
// collector clear lets a known gossip in again, GossipProtocolImpl.java:205-213 with :217-236) lives
// in the member's infected-overflow table, keyed by (gossiper, seq), so it does not move when the
// sweep compacts the slab.
constexpr uint32_t PER_BITS = 28, PER_MASK = (1u << PER_BITS) - 1;  // infection period: 2^28 rounds
struct alignas(16) GossipHot {
  uint32_t gossiper, seq;
  uint32_t per_st;  // infection period (bits 0..27) | status << 28 (3 bits) | more << 31: inf[1..] in use
  uint32_t inf0;    // GossipState.infected's first member (the first sender), NONE = empty
  __device__ __forceinline__ uint32_t inf_period() const { return per_st & PER_MASK; }
  __device__ __forceinline__ uint32_t status() const { return (per_st >> PER_BITS) & 7u; }
  __device__ __forceinline__ bool more() const { return (per_st >> 31) != 0; }
};
struct alignas(8) GossipCold {
  uint32_t subject;  // the record's member, or a user gossip's payload handle
  int32_t inc;
};
static_assert(sizeof(GossipHot) == 16 && sizeof(GossipCold) == 8, "24 B per GossipState");
// infected-overflow entry: GossipState.infected[1..] of one (gossiper, seq) of one member
constexpr uint32_t INF_EMPTY = 0xffffffffu;  // gossiper value of a free slot
struct alignas(16) InfOver {
  uint32_t gossiper, seq;
  uint32_t inf[GINF - 1];
  uint32_t pad;
};
static_assert(sizeof(InfOver) == 32, "32 B per infected overflow");
// linear probing from the key's hash; a lookup stops at an empty slot.  An entry is removed by
// backward-shift deletion (inf_erase: the entries after it on its probe run move up), so the table
// holds no tombstones and a miss stops at the first free slot however long the run has been going.
// One writer per member at a time, one lane at a time: its delivery's serial steps, or one lane of
// its sender wave's sweep after another (emit_one), with no reader of the table in between.
__device__ __forceinline__ uint32_t inf_hash(uint32_t g, uint32_t q) { return (g * 0x9e3779b1u) ^ (q * 0x85ebca77u); }
__device__ inline int32_t inf_find(const InfOver* t, uint32_t mask, uint32_t g, uint32_t q) {
  for (uint32_t i = 0, h = inf_hash(g, q) & mask; i <= mask; ++i, h = (h + 1) & mask) {
    const uint32_t k = t[h].gossiper;
    if (k == INF_EMPTY) return -1;
    if (k == g && t[h].seq == q) return (int32_t)h;
  }
  return -1;
}
// frees slot f: each later entry of the run whose home slot does not lie cyclically in (hole, its
// slot] moves into the hole, until a free slot ends the run
__device__ inline void inf_erase(InfOver* t, uint32_t mask, uint32_t f) {
  uint32_t hole = f;
  for (uint32_t n = 0, j = (f + 1) & mask; n < mask; ++n, j = (j + 1) & mask) {
    const InfOver x = t[j];
    if (x.gossiper == INF_EMPTY) break;
    const uint32_t h = inf_hash(x.gossiper, x.seq) & mask;
    const bool stays = hole <= j ? (h > hole && h <= j) : (h > hole || h <= j);
    if (!stays) {
      t[hole] = x;
      hole = j;
    }
  }
  t[hole].gossiper = INF_EMPTY;
}
// lane l's value to every lane when l is wave-uniform: v_readlane (a register read) instead of the
// LDS crossbar round trip __shfl takes
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, uint32_t l) {
  return (uint64_t)rdlane((uint32_t)v, l) | ((uint64_t)rdlane((uint32_t)(v >> 32), l) << 32);
}
// a load through the global address space (global_load: counted by vmcnt only, while a generic-pointer
// flat load also holds lgkmcnt, so an LDS-only wait would wait for it too)
template <typename T>
__device__ __forceinline__ T gload(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass of hipcc has no address space 1; it never runs this)
  typedef const __attribute__((address_space(1))) T* gptr;
  return *(gptr)(p);
#else
  return *p;
#endif
}
struct SlabRef {
  GossipHot* hot;
  GossipCold* cold;
  InfOver* inf;      // the member's infected-overflow table
  uint32_t inf_mask;
  uint32_t* err;
  uint32_t base, mask;  // ring: gossip p at (base + p) & mask
  __device__ __forceinline__ GossipHot& H(uint32_t p) const { return hot[(base + p) & mask]; }
  __device__ __forceinline__ GossipCold& C(uint32_t p) const { return cold[(base + p) & mask]; }
  __device__ __forceinline__ GossipHot Hg(uint32_t p) const { return gload(hot + ((base + p) & mask)); }
  __device__ __forceinline__ GossipDev get(uint32_t p) const {
    const GossipHot h = H(p);
    const GossipCold k = C(p);
    GossipDev g;
    g.gossiper = h.gossiper;
    g.seq = h.seq;
    g.inf_period = h.inf_period();
    g.status = h.status();
    g.subject = k.subject;
    g.inc = k.inc;
    g.inf[0] = h.inf0;
#pragma unroll
    for (int i = 1; i < GINF; ++i) g.inf[i] = NONE;
    if (h.more()) {
      const int32_t f = inf_find(inf, inf_mask, h.gossiper, h.seq);
      if (f >= 0)
#pragma unroll
        for (int i = 1; i < GINF; ++i) g.inf[i] = inf[f].inf[i - 1];
    }
    return g;
  }
  __device__ __forceinline__ void put(uint32_t p, const GossipDev& g) const {
    GossipHot h;
    h.gossiper = g.gossiper;
    h.seq = g.seq;
    const bool more = g.inf[1] != NONE;
    h.per_st = (g.inf_period & PER_MASK) | (g.status << PER_BITS) | (more ? 1u << 31 : 0u);
    h.inf0 = g.inf[0];
    GossipCold k;
    k.subject = g.subject;
    k.inc = g.inc;
    if (more) {
      int32_t f = inf_find(inf, inf_mask, g.gossiper, g.seq);
      if (f < 0) {  // a new entry: the first free slot on the probe path
        for (uint32_t i = 0, x = inf_hash(g.gossiper, g.seq) & inf_mask; i <= inf_mask; ++i, x = (x + 1) & inf_mask)
          if (inf[x].gossiper == INF_EMPTY) { f = (int32_t)x; break; }
      }
      if (f < 0) {
        atomicOr(err, ERR_INFECTED);  // the member's overflow table is full
      } else {
        InfOver o;
        o.gossiper = g.gossiper;
        o.seq = g.seq;
#pragma unroll
        for (int i = 1; i < GINF; ++i) o.inf[i - 1] = g.inf[i];
        o.pad = 0;
        inf[f] = o;
      }
    }
    H(p) = h;
    C(p) = k;
  }
  // the sweep dropped a state whose infected list overflowed (one lane of the wave at a time)
  __device__ __forceinline__ void drop_more(uint32_t g, uint32_t q) const {
    const int32_t f = inf_find(inf, inf_mask, g, q);
    if (f >= 0) inf_erase(inf, inf_mask, (uint32_t)f);
  }
};

// SequenceIdCollector (SequenceIdCollector.java) of (viewer, gossiper), 16 B: a collector holds one
// interval almost always (a gossiper's sequence ids reach a member in order), so the interval is
// inline.  One that needs more (out-of-order arrival, loss) spills to a block of a size tier —
// 6, 62, 510 or 16,382 closed intervals (64 B .. 128 KiB: a 4-word header {count} + (lo, hi) pairs,
// ascending) — grows tier by tier, and returns inline when its intervals merge back into one.
// The reference keeps up to gossipSegmentationThreshold (1,000) intervals before a gossip round
// clears the collector (checkGossipSegmentation, GossipProtocolImpl.java:217-236); the top tier
// leaves room for a round's growth beyond that.  Freed blocks are recycled from the next tick on.
struct alignas(16) CollEnt {
  uint32_t key;   // gossiper + 1; 0 = empty slot
  uint32_t lo, hi;
  uint32_t meta;  // bits 0..2: inline interval count (0 / 1) or COLL_SPILLED; bit 3: cleared;
                  // bits 4..5: spill tier; bits 8..31: block index in the tier
};
constexpr uint32_t COLL_SPILLED = 7u, COLL_CLEARED = 8u;
__host__ __device__ constexpr uint32_t tier_cap(int t) { return t == 0 ? 6u : t == 1 ? 62u : t == 2 ? 510u : 16382u; }
__host__ __device__ constexpr uint32_t tier_words(int t) { return 4u + 2u * tier_cap(t); }
struct SpillCtl {  // one per tier
  uint32_t bump;    // blocks ever carved from the pool
  int32_t avail;    // recyclable blocks in `avail` (may dip below 0 during a tick: failed pops)
  uint32_t freed;   // blocks freed this tick (recyclable from the next)
  uint32_t pad;
};

struct LinkDev {  // NetworkEmulator per-link override, sorted by (a, b)
  uint32_t a, b;
  int32_t out_loss;   // outboundSettings(b) on a; -1 = none
  int32_t in_pass;    // inboundSettings(b) on a (a receives from b); -1 = none
  int32_t out_delay;  // outboundSettings(b).meanDelay on a as a delay-table index; -1 = none, -2 = 0 ms
};

// A GOSSIP_REQ in flight: 32 B, two 16-B stores by the sender, two 16-B loads by the receiver.
struct alignas(16) GMsgFull {
  uint32_t to;       // the receiver, until the message is in its inbox; there: its age in ticks
                     // (a message the network emulator delayed, 0 otherwise)
  uint32_t from;     // the sender (GossipRequest.from)
  uint32_t gossiper, seq, subject;  // Gossip id and the record (or user payload handle) it carries
  uint32_t inc_st;   // incarnation (bits 0..28) | status << 29
  uint32_t pos_dup;  // the sender's slab position (bits 0..30) | dup << 31: the receiver's collector
                     // already held the sequence id on arrival (a no-op)
  uint32_t pseq;     // place among the round's messages of the (from, to) pair in slab-position order;
                     // in the delay ring: the sending tick, until k_dq_release ranks it
  __device__ __forceinline__ int32_t inc() const { return (int32_t)(inc_st & 0x1fffffffu); }
  __device__ __forceinline__ uint32_t status() const { return inc_st >> 29; }
  __device__ __forceinline__ uint32_t pos() const { return pos_dup & 0x7fffffffu; }
  __device__ __forceinline__ bool dup() const { return (pos_dup >> 31) != 0; }
  __device__ __forceinline__ void set_gossip(uint32_t g, uint32_t q, uint32_t subj, uint32_t st, int32_t inc) {
    gossiper = g;
    seq = q;
    subject = subj;
    inc_st = ((uint32_t)inc & 0x1fffffffu) | (st << 29);
  }
};
static_assert(sizeof(GMsgFull) == 32, "a GOSSIP_REQ is two 16-B words");

struct SyncReq {  // SYNC (request) or SYNC_ACK
  uint32_t from, to, ordinal, slot;
  uint32_t flags;    // bit0 initial, bit1 outfail, bit2 delivered; bits 8..31 record count (RQ_RECS_SHIFT)
  uint32_t content;  // NONE: `from` is owned here (row / snapshot); else index into the received rows
  uint32_t snap;     // k_sync_prep: snapshot slot of `from`'s row in this sub-phase, or NONE
  uint32_t pad;
};

struct InsOp {  // deferred pingMembers.add(nextInt(size), member) of an ADDED event
  uint32_t s, phase, minor, next;  // next: the viewer's following op in event order (chain)
};
// a viewer's first INS_INLINE ops of a phase sit in its own slots (read in parallel by the list
// kernel); later ones go to blocks of the shared op array — 8, 16, 32, 64, 128, then 256 ops, each
// block reserved whole when its first op comes (the one thread that owns the viewer in the phase
// appends them).  The first op of a block holds the next block's start in `next`: the list kernel
// hops block to block and reads a batch's ops in parallel, where an op-by-op chain took one
// dependent load per op (16 K for a joiner's initial SYNC_ACK).
constexpr uint32_t INS_INLINE = 8;
// block of beyond-inline op j: its index, j's offset in it and its size
__device__ __forceinline__ uint32_t ins_block_of(uint32_t j, uint32_t& off, uint32_t& size) {
  if (j < 248) {
    const uint32_t b = 31u - (uint32_t)__clz(j / 8 + 1);
    off = j - 8 * ((1u << b) - 1);
    size = 8u << b;
    return b;
  }
  off = (j - 248) % 256;
  size = 256;
  return 5 + (j - 248) / 256;
}

// Receipt bitmap slot: gossip (gossiper, seq) hashes to one of GSLOTS slots; the slot's bits are
// valid for the gossip `key` from tick `tick` on (a slot is (re)claimed only in k_end_tick, when no
// other kernel runs, and its bits are zeroed then).
constexpr uint32_t GSLOTS = 8192;
// The bits are receiver-major: receiver i's row is GROW words (1 KB), bit sl of it says i accepted
// slot sl's gossip.  The checks come a receiver at a time: emit tests a sender's few targets against
// the 64 gossips of a pass (at most 8 lines of each target's row, where a gossip-major layout reads a
// line per (gossip, target)), and delivery marks one receiver's accepted lanes into one row.  A claim
// clears one bit of every row (k_end_tick); claims are per new gossip, a few hundred per run.
constexpr uint32_t GROW = GSLOTS / 32;
constexpr uint32_t GSLOT_HOLD = 64;  // ticks a claimed slot stays with its gossip before another may take it
__device__ __forceinline__ size_t rbit_word(uint32_t i, uint32_t sl) { return (size_t)i * GROW + (sl >> 5); }
struct GSlot {
  uint64_t key;   // (gossiper + 1) << 32 | seq, 0 = unowned
  uint32_t tick;  // bits set from this tick on are trustworthy
  uint32_t pad;
};
__device__ __forceinline__ uint64_t gkey(uint32_t gossiper, uint32_t seq) {
  return ((uint64_t)(gossiper + 1) << 32) | seq;
}
__device__ __forceinline__ uint32_t gslot_of(uint64_t key) {
  uint64_t x = key * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(x >> 51) & (GSLOTS - 1);  // 13 bits
}

// Row sharding: shard r owns viewers [lo, lo + nl) with lo = r * sz.  Every array
// indexed by viewer (cells, lists, slab, collectors, mem, per-viewer counters) holds owned rows only
// and is indexed by v - lo; the network emulator, seeds and `up` are replicated.
struct Ctx {
  uint32_t n, gcap, hcap, wheel_mask, wheel_nq;
  uint32_t lo, nl, sz, rank, world;
  uint32_t xchg;  // the exchange machinery is on: world > 1, or an RCCL engine of one rank (swim.h)
  uint32_t P, to_ticks, relay_ticks, G, S, sync_to_ticks, tick_ms;
  uint32_t metadata_timeout;  // ms (a delayed GET_METADATA round trip must finish before it)
  int32_t ping_interval, suspicion_mult, repeat_mult, fanout, ping_req_members, seg_threshold, record_fd;
  uint32_t key0, key1;
  uint64_t T;
  // the view cell of (viewer, subject) is stored split in two u32 words (layout below)
  uint32_t* recs;  // [nl][n] MembershipRecord: what SYNC carries and the merge filter reads
  uint32_t* aux;   // [nl][n] the viewer-local side maps (members / aliveEmitted / metadata / timer)
  // exact block witness of the record rows: ref is this shard's reference record per
  // subject, bdiff[row][blk] the number of subjects of 1,024-subject block blk whose record in the row
  // differs from ref — two rows with bdiff 0 in a block hold identical records there.  Maintained on
  // every record write (cell_put); ref follows the rows' majority (k_end_tick's rebase of the subjects
  // marked dirty).
  uint32_t* ref;     // [n]
  uint32_t* bdiff;   // [nl][blocks]
  uint32_t* bnz;     // [nl] blocks of the row whose bdiff is non-zero (the quiet scan's O(1) row check)
  uint32_t* dirty;   // [n] 1: some row's record of the subject changed since the last rebase
  uint32_t blocks;   // ceil(n / 1024)
  MemberDev* mem;
  uint8_t* up;  // replicated: member's transport is running
  // replicated (swim_join_at): route[x] = the member listening on member x's address now; nullptr
  // while every member listens on its own address
  const uint32_t* route;
  uint32_t* ping;
  uint32_t* remote;
  GossipHot* slab_hot;   // [nl][gcap] (SlabRef)
  GossipCold* slab_cold;  // [nl][gcap]
  InfOver* inf_over;      // [nl][inf_mask + 1] GossipState.infected beyond the first member
  uint32_t inf_mask;
  uint32_t* gix;       // [nl][gix_mask + 1] slab serials by (gossiper, seq), open addressing
  uint32_t gix_mask;
  CollEnt* coll;       // [nl][hcap] open addressing by gossiper
  uint32_t* spill[NTIER];        // spilled collectors: tier t holds spill_cap[t] blocks of tier_words(t)
  uint32_t* spill_avail[NTIER];  // recyclable block indices
  uint32_t* spill_freed[NTIER];  // block indices freed this tick
  uint32_t spill_cap[NTIER];
  SpillCtl* spill_ctl;           // [NTIER]
  uint32_t* seg_flag;            // per viewer: a collector exceeded gossipSegmentationThreshold
  uint32_t* fd_sync;
  // suspicion-timer wheel: one queue per (deadline bucket, 256-viewer block), paged.  Queue q of
  // bucket b holds wheel_cnt[b][q] entries (viewer << 32 | subject); entry i lives in page
  // wheel_pt[b][q][i >> wheel_pshift], slot i & page mask.  Pages come from a shared pool (bump +
  // recycled: pages of a bucket fired this tick are reusable from the next), so the wheel holds
  // timer_capacity entries in all buckets together, however they cluster in time (a partition
  // schedules N/2 timers at every viewer within a few ticks).
  uint64_t* wheel;      // [wheel_pages][1 << wheel_pshift]
  uint32_t* wheel_cnt;  // [W][wheel_nq]
  uint32_t* wheel_pt;   // [W][wheel_nq][wheel_ptmax] page ids (NONE = not allocated yet)
  uint32_t* wheel_avail;  // recyclable page ids
  uint32_t* wheel_freed;  // page ids freed this tick
  SpillCtl* wheel_ctl;    // {bump, avail, freed}
  uint32_t wheel_pages, wheel_ptmax, wheel_pshift;  // page: 64 .. 4,096 entries (host-sized)
  swim_event* ev;
  uint32_t* ev_cnt;     // [SUBQ]
  uint32_t ev_cap;      // per sub-queue
  // network emulator
  uint8_t* default_loss;
  uint8_t* default_inbound;
  uint16_t* group;
  uint32_t partition;
  LinkDev* links;
  uint32_t n_links;
  // message delay (swim_delay.h): thresholds per distinct meanDelay, the default table of each
  // member (-1 = no delay); delay_on: some member or link has a delay
  // namespaces (areNamespacesRelated, MembershipProtocolImpl.java:511-536): group of each member,
  // relation matrix of the groups; n_ns = 0: one namespace
  const uint16_t* ns;
  const uint8_t* ns_rel;
  uint32_t n_ns;
  // metadata version of each member (replicated; ClusterImpl.updateMetadata bumps it) and, once a
  // metadata update happened, the version each owned viewer's MetadataStore holds per subject
  uint32_t* meta_ver;
  uint32_t* meta_seen;  // [nl][n] or nullptr
  const uint64_t* delay_th;  // [tables][SWIM_DELAY_TICKS_MAX]
  int16_t* default_delay;    // replicated [n]
  uint32_t delay_on;
  // delayed metadata round trips (allocated with the delay machinery): entries [2][fq_cap] and
  // per-viewer chain heads / tails [2][nl] by tick parity, entry counts [2]
  FetchEnt* fq;
  uint32_t* fq_head;
  uint32_t* fq_tail;
  uint32_t* fq_cnt;
  uint32_t fq_cap;
  PAck* pa;        // [nl][pa_cap] PendingAcks, creation order
  uint32_t* pa_n;  // [nl]
  uint32_t pa_cap;
  uint8_t* is_seed;
  uint32_t* seeds;
  uint32_t n_seeds;
  // per-member seedMembers (swim_set_member_seeds), replicated: member v with mseed_own[v] uses
  // mseed[mseed_off[v] .. mseed_off[v + 1]) instead of the engine-wide list; nullptr: nobody does
  const uint8_t* mseed_own;
  const uint32_t* mseed_off;
  const uint32_t* mseed;
  // deferred list ops: a viewer's ops of one phase are applied by whoever delivered to it, right
  // after its deliveries / merges (k_gossip_deliver, k_sync_apply)
  InsOp* ins;              // overflow chain storage, shared by the viewers of the phase
  InsOp* ins_inline;       // [nl][INS_INLINE] each viewer's first ops of the phase
  uint32_t* ins_total;
  uint32_t ins_cap;
  uint32_t* compact_flag;  // per viewer: lists hold a REMOVED member (compacted before its next FD step)
  // compact per-member schedule: lets the per-tick member scans skip idle members
  // without touching their MemberDev
  uint32_t* fd_next;    // next tick with FD work (ping due, ack or relay timeout); stale while down
  uint32_t* sync_next;  // next periodic-SYNC tick (NONE: periodic SYNC off)
  uint32_t* mflag;      // MF_* work for SYNC collection / k_end_tick
  GossipSched* gs;      // per member: gossip round schedule, period and slab length (one 16-B word)
  // receipt bitmaps: a subset of "receiver t's collector holds gossip (gossiper, seq)"
  // that k_gossip_emit tests before probing the collector table
  GSlot* gslot;          // [GSLOTS] the gossip owning each bitmap and the tick its bits became valid
  uint64_t* gpend;       // [GSLOTS] gossip waiting to own the slot at the end of the tick (0 = none)
  uint32_t* gbits;       // [nl][GROW] bit sl of row t - lo: receiver t accepted slot sl's owning gossip
  uint32_t* clr_tick;    // per viewer: last tick one of its collectors was cleared
  uint32_t* gclaim;      // [2][GSLOTS] slots to (re)claim at the end of tick T, queue T & 1
  uint32_t* gclaim_cnt;  // [2]
  unsigned long long* stats;
  uint32_t* err;
};

// ------------------------------------------------------------------------------- Philox4x32-10
__device__ __forceinline__ uint32_t philox_w0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c0;
}

__device__ __forceinline__ void philox4(const uint32_t in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

__device__ __forceinline__ uint32_t draw_at(const Ctx& c, uint32_t member, uint64_t tick, uint32_t stream,
                                            uint32_t sub24, uint32_t sub32) {
  return philox_w0(member, (uint32_t)tick, (stream << 24) | (sub24 & 0xffffffu), sub32, c.key0, c.key1);
}
__device__ __forceinline__ uint32_t draw(const Ctx& c, uint32_t member, uint32_t stream, uint32_t sub24, uint32_t sub32) {
  return draw_at(c, member, c.T, stream, sub24, sub32);
}
__device__ __forceinline__ uint32_t next_int(uint32_t w, uint32_t bound) {
  return (uint32_t)(((uint64_t)w * bound) >> 32);
}
__device__ __forceinline__ bool lost(int32_t pct, uint32_t w) {
  return pct > 0 && (pct >= 100 || (int32_t)next_int(w, 100) < pct);
}

// ------------------------------------------------------------------------------- cells
__device__ __forceinline__ int32_t c_inc(uint64_t c) { return (int32_t)(uint32_t)c; }
__device__ __forceinline__ uint32_t c_status(uint64_t c) { return (uint32_t)((c >> 32) & 3u); }
__device__ __forceinline__ bool c_has(uint64_t c, uint64_t b) { return (c & b) != 0; }
__device__ __forceinline__ uint32_t c_deadline(uint64_t c) { return (uint32_t)(c >> 39); }
__device__ __forceinline__ uint64_t c_with_record(uint64_t c, uint32_t st, int32_t inc) {
  return (c & ~0x3ffffffffull) | (uint64_t)(uint32_t)inc | ((uint64_t)st << 32);
}
__device__ __forceinline__ uint64_t c_with_deadline(uint64_t c, uint64_t tick) {
  return (c & ((1ull << 39) - 1)) | ((tick & SWIM_DEADLINE_MASK) << 39);
}
__device__ __forceinline__ void set_err(const Ctx& c, uint32_t bit) { atomicOr(c.err, bit); }

// ---- split cell storage.  The swim.h packed u64 cell stays the logical format
// (cell_get / cell_put); the hot SYNC stream touches only the record words.
//   rec: bits 0..28 incarnation (0 .. 2^29-2, else ERR_INC), 29..30 status, 31 in_table
//   aux: bit 0 in_members, 1 alive_emitted, 2 has_timer, 3 has_metadata, 4..28 timer deadline
constexpr uint32_t REC_INC_MASK = 0x1fffffffu;
constexpr uint32_t REC_IN_TABLE = 0x80000000u;
constexpr uint32_t A_IN_MEMBERS = 1u, A_ALIVE_EMITTED = 2u, A_HAS_TIMER = 4u, A_HAS_METADATA = 8u;
__device__ __forceinline__ int32_t r_inc(uint32_t r) { return (int32_t)(r & REC_INC_MASK); }
__device__ __forceinline__ uint32_t r_status(uint32_t r) { return (r >> 29) & 3u; }
__device__ __forceinline__ bool r_in_table(uint32_t r) { return (r & REC_IN_TABLE) != 0; }
__device__ __forceinline__ uint32_t* rec_row(const Ctx& c, uint32_t v) { return c.recs + (size_t)(v - c.lo) * c.n; }
__device__ __forceinline__ uint32_t* aux_row(const Ctx& c, uint32_t v) { return c.aux + (size_t)(v - c.lo) * c.n; }
__device__ __forceinline__ uint64_t compose_cell(uint32_t r, uint32_t a) {
  return (uint64_t)(r & REC_INC_MASK) | ((uint64_t)r_status(r) << 32) | ((uint64_t)(r >> 31) << 34) |
         ((uint64_t)(a & 0xfu) << 35) | ((uint64_t)(a >> 4) << 39);
}
__device__ __forceinline__ uint64_t cell_get(const Ctx& c, uint32_t v, uint32_t s) {
  const size_t i = (size_t)(v - c.lo) * c.n + s;
  return compose_cell(c.recs[i], c.aux[i]);
}
constexpr uint32_t BLK_SHIFT = 10;  // 1,024-subject blocks (= the SYNC classify unit)
// bdiff[row][blk] += d (d = +-1), and the row's count of non-zero blocks follows the 0 <-> 1
// transitions.  Each atomic returns a distinct old value, so the transitions of one block alternate
// in atomic order and bnz is exact once the kernel's updates have all completed.
__device__ __forceinline__ void bdiff_add(const Ctx& c, uint32_t row, uint32_t blk, int d) {
  const uint32_t old = atomicAdd(&c.bdiff[(size_t)row * c.blocks + blk], (uint32_t)d);
  if (d > 0 && old == 0u) atomicAdd(&c.bnz[row], 1u);
  else if (d < 0 && old == 1u) atomicSub(&c.bnz[row], 1u);
}
// the block witness follows a record change of (v, s): old -> nr (atomic: a row's cells may change
// from several threads of one kernel, e.g. entry-parallel timers)
__device__ inline void rec_changed(const Ctx& c, uint32_t v, uint32_t s, uint32_t old, uint32_t nr) {
  const uint32_t rf = c.ref[s];
  const int d = (nr != rf ? 1 : 0) - (old != rf ? 1 : 0);
  if (d) bdiff_add(c, v - c.lo, s >> BLK_SHIFT, d);
  c.dirty[s] = 1u;
}
__device__ __forceinline__ void cell_put(const Ctx& c, uint32_t v, uint32_t s, uint64_t cell) {
  const size_t i = (size_t)(v - c.lo) * c.n + s;
  const uint32_t inc = (uint32_t)cell;
  if (inc >= REC_INC_MASK) set_err(c, ERR_INC);
  const uint32_t nr = (inc & REC_INC_MASK) | ((uint32_t)((cell >> 32) & 3u) << 29) | ((uint32_t)((cell >> 34) & 1u) << 31);
  const uint32_t old = c.recs[i];
  c.recs[i] = nr;
  c.aux[i] = (uint32_t)((cell >> 35) & 0xfu) | ((uint32_t)((cell >> 39) & SWIM_DEADLINE_MASK) << 4);
  if (nr != old) rec_changed(c, v, s, old, nr);
}
__device__ __forceinline__ MemberDev& mem(const Ctx& c, uint32_t v) { return c.mem[v - c.lo]; }
__device__ __forceinline__ GossipSched& gsched(const Ctx& c, uint32_t v) { return c.gs[v - c.lo]; }
__device__ __forceinline__ uint32_t* ping_list(const Ctx& c, uint32_t v) { return c.ping + (size_t)(v - c.lo) * c.n; }
__device__ __forceinline__ uint32_t* remote_list(const Ctx& c, uint32_t v) { return c.remote + (size_t)(v - c.lo) * c.n; }
__device__ __forceinline__ SlabRef slab_of(const Ctx& c, uint32_t v, uint32_t base) {
  const size_t o = (size_t)(v - c.lo) * c.gcap;
  return SlabRef{c.slab_hot + o, c.slab_cold + o, c.inf_over + (size_t)(v - c.lo) * (c.inf_mask + 1), c.inf_mask, c.err,
                 base, c.gcap - 1};
}
__device__ __forceinline__ SlabRef slab_of(const Ctx& c, uint32_t v) { return slab_of(c, v, c.gs[v - c.lo].base); }
__device__ __forceinline__ bool owned(const Ctx& c, uint32_t v) { return v - c.lo < c.nl; }
__device__ __forceinline__ uint32_t owner(const Ctx& c, uint32_t v) { return v / c.sz; }

// Counters are replicated ST_REPL times (summed on readback) so that thousands of workgroups never
// serialise on one address (MI355X_MICROARCH.md: one contended address is ~14x slower).
constexpr int ST_REPL = 64;
__device__ __forceinline__ void stat_add(const Ctx& c, int slot, unsigned long long x) {
  if (x) atomicAdd(&c.stats[slot * ST_REPL + (blockIdx.x & (ST_REPL - 1))], x);
}
// wave-reduced counter add; every lane of the wave must be active (call after reconvergence)
__device__ __forceinline__ void wave_stat_add(const Ctx& c, int slot, unsigned long long x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
  if ((threadIdx.x & 63) == 0) stat_add(c, slot, x);
}

// MembershipRecord.isOverrides (MembershipRecord.java:67-88); r0p = false for "no record"
__device__ __forceinline__ bool is_overrides(uint32_t s1, int32_t i1, bool r0p, uint32_t s0, int32_t i0) {
  if (!r0p) return s1 == SWIM_ALIVE || s1 == SWIM_LEAVING;
  if (s1 == s0 && i1 == i0) return false;
  if (s0 == SWIM_DEAD) return false;
  if (s1 == SWIM_DEAD) return true;
  if (i1 == i0) return s1 == SWIM_SUSPECT && (s0 == SWIM_ALIVE || s0 == SWIM_LEAVING);
  return i1 > i0;
}

// ------------------------------------------------------------------------------- network emulator
__device__ __forceinline__ const LinkDev* find_link(const Ctx& c, uint32_t a, uint32_t b) {
  uint32_t lo = 0, hi = c.n_links;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    const LinkDev& L = c.links[mid];
    if (L.a < a || (L.a == a && L.b < b)) lo = mid + 1; else hi = mid;
  }
  if (lo < c.n_links && c.links[lo].a == a && c.links[lo].b == b) return &c.links[lo];
  return nullptr;
}
// NetworkEmulator.outboundSettings(dst) on src (NetworkEmulator.java:59-61)
__device__ __forceinline__ int32_t out_loss(const Ctx& c, uint32_t a, uint32_t b) {
  if (c.partition && c.group[a] != c.group[b]) return 100;
  if (c.n_links) {
    const LinkDev* L = find_link(c, a, b);
    if (L && L->out_loss >= 0) return L->out_loss;
  }
  return c.default_loss[a];
}
// NetworkEmulator.inboundSettings(src).shallPass() on receiver b (NetworkEmulator.java:212-214)
__device__ __forceinline__ bool in_pass(const Ctx& c, uint32_t b, uint32_t a) {
  if (c.n_links) {
    const LinkDev* L = find_link(c, b, a);
    if (L && L->in_pass >= 0) return L->in_pass != 0;
  }
  return c.default_inbound[b] != 0;
}
// tryDelayOutbound (NetworkEmulator.java:190-202) + evaluateDelay (:359-369) of a message a -> b, in
// ticks (swim_delay.h); the draw is keyed (member, stream, sub24, sub32) and taken only when the
// link has a mean delay
__device__ inline uint32_t delay_ticks(const Ctx& c, uint32_t a, uint32_t b, uint32_t member, uint32_t stream,
                                       uint32_t sub24, uint32_t sub32) {
  if (!c.delay_on) return 0;
  int32_t tab = c.default_delay[a];
  if (c.n_links) {
    const LinkDev* L = find_link(c, a, b);
    if (L && L->out_delay != -1) tab = L->out_delay;
  }
  if (tab < 0) return 0;
  const uint32_t in[4] = {member, (uint32_t)c.T, (stream << 24) | (sub24 & 0xffffffu), sub32};
  uint32_t o[4];
  philox4(in, c.key0, c.key1, o);
  const uint64_t u53 = ((uint64_t)(o[0] >> 11) << 32) | o[1];
  return swim_delay_ticks(c.delay_th + (size_t)tab * SWIM_DELAY_TICKS_MAX, u53);
}
// lost() with the Philox draw evaluated only when the loss percentage needs it (0 % and 100 %
// are decided without a draw; draws are keyed, so skipping one shifts nothing)
__device__ __forceinline__ bool lost_k(const Ctx& c, int32_t pct, uint32_t member, uint32_t stream, uint32_t sub24,
                                       uint32_t sub32) {
  if (pct <= 0) return false;
  if (pct >= 100) return true;
  return (int32_t)next_int(draw(c, member, stream, sub24, sub32), 100) < pct;
}
// tryFailOutbound (NetworkEmulator.java:167-181) + a stopped destination refusing the connection;
// the draw is keyed (member, stream, sub24, sub32)
// the member a message sent to x's address reaches (Transport.send / requestResponse by Address)
__device__ __forceinline__ uint32_t dst(const Ctx& c, uint32_t x) { return c.route ? c.route[x] : x; }

__device__ __forceinline__ bool out_fail(const Ctx& c, uint32_t a, uint32_t b, uint32_t member, uint32_t stream,
                                         uint32_t sub24, uint32_t sub32) {
  return !c.up[b] || lost_k(c, out_loss(c, a, b), member, stream, sub24, sub32);
}

// ------------------------------------------------------------------------------- collectors
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// Linear probing, four slots per round trip: a round loads the keys of the next four slots of the
// probe sequence together (a loaded table's runs are long: one dependent load per slot made the
// storm's collector lookups the deepest chains of the delivery and fanout kernels), then takes the
// first that matches or is empty, in probe order — the same slot a one-by-one probe finds.
__device__ inline CollEnt* coll_find(const Ctx& c, uint32_t v, uint32_t gossiper) {
  CollEnt* base = c.coll + (size_t)(v - c.lo) * c.hcap;
  uint32_t mask = c.hcap - 1, h = hash32(gossiper) & mask, key = gossiper + 1;
  for (uint32_t i = 0; i < c.hcap; i += 4) {
    uint32_t k[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) k[q] = base[(h + i + q) & mask].key;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (k[q] == key) return base + ((h + i + q) & mask);
      if (k[q] == 0) return nullptr;
    }
  }
  return nullptr;
}
// ensureSequence (GossipProtocolImpl.java:279-281)
__device__ inline CollEnt* coll_ensure(const Ctx& c, uint32_t v, uint32_t gossiper) {
  CollEnt* base = c.coll + (size_t)(v - c.lo) * c.hcap;
  uint32_t mask = c.hcap - 1, h = hash32(gossiper) & mask, key = gossiper + 1;
  for (uint32_t i = 0; i < c.hcap; ++i) {
    CollEnt* e = base + ((h + i) & mask);
    if (e->key == key) return e;
    if (e->key == 0) {
      e->key = key;
      e->lo = e->hi = 0;
      e->meta = 0;
      return e;
    }
  }
  set_err(c, ERR_HASH);
  return nullptr;
}
// coll_ensure that also returns the entry's value (each probe one 16-B load; a new entry is the
// value it was initialised with)
__device__ inline CollEnt* coll_ensure_v(const Ctx& c, uint32_t v, uint32_t gossiper, CollEnt& out) {
  CollEnt* base = c.coll + (size_t)(v - c.lo) * c.hcap;
  uint32_t mask = c.hcap - 1, h = hash32(gossiper) & mask, key = gossiper + 1;
  for (uint32_t i = 0; i < c.hcap; ++i) {
    CollEnt* e = base + ((h + i) & mask);
    const CollEnt x = *e;
    if (x.key == key) { out = x; return e; }
    if (x.key == 0) {
      CollEnt ne;
      ne.key = key; ne.lo = 0; ne.hi = 0; ne.meta = 0;
      *e = ne;
      out = ne;
      return e;
    }
  }
  set_err(c, ERR_HASH);
  return nullptr;
}
// coll_ensure_v for the leader lanes of one wave (lead: one per distinct gossiper) inserting into one
// member's table that no other wave touches meanwhile: two leaders finding the same empty slot are
// told apart by ballot (the lowest lane takes it, the others probe on), so no compare-and-swap round
// trip.  Called by the whole wave; returns the leader's entry (null: not a leader, or the table is full).
__device__ inline CollEnt* coll_ensure_wave(const Ctx& c, uint32_t v, bool lead, uint32_t gossiper, uint32_t lane,
                                            CollEnt& out, uint32_t* probes = nullptr) {
  CollEnt* base = c.coll + (size_t)(v - c.lo) * c.hcap;
  const uint32_t mask = c.hcap - 1, key = gossiper + 1;
  uint32_t h = hash32(gossiper) & mask;
  CollEnt* res = nullptr;
  bool act = lead;
  // a round: the entry at h and the keys of the three slots after it, in one round trip; a match
  // among those three moves h onto it (its entry comes with the next round), an empty one is claimed
  for (uint32_t it = 0; __ballot(act); ++it) {
    if (probes) ++*probes;
    if (it == c.hcap) {  // (wave-uniform)
      if (act) set_err(c, ERR_HASH);
      break;
    }
    CollEnt x{};
    uint32_t k1 = 0, k2 = 0, k3 = 0;
    if (act) {
      x = base[h];
      k1 = base[(h + 1) & mask].key;
      k2 = base[(h + 2) & mask].key;
      k3 = base[(h + 3) & mask].key;
    }
    if (act && x.key == key) {
      out = x;
      res = base + h;
      act = false;
    }
    // the first of the four slots that matches or is empty (4: none)
    const uint32_t q = x.key == 0 ? 0u : k1 == key || k1 == 0 ? 1u : k2 == key || k2 == 0 ? 2u : k3 == key || k3 == 0 ? 3u : 4u;
    const uint32_t kq = q == 1u ? k1 : q == 2u ? k2 : k3;
    const bool claim = act && q < 4u && (q == 0u || kq == 0u);
    const uint32_t slot = (h + q) & mask;
    bool won = false;
    for (uint64_t todo = __ballot(claim); todo;) {
      const uint32_t l = (uint32_t)__ffsll((unsigned long long)todo) - 1;
      const uint32_t sl = rdlane(slot, l);
      todo &= ~__ballot(claim && slot == sl);
      won |= lane == l;
    }
    if (won) {
      CollEnt ne;
      ne.key = key; ne.lo = 0; ne.hi = 0; ne.meta = 0;
      base[slot] = ne;
      out = ne;
      res = base + slot;
      act = false;
    }
    // on: onto the match, past a slot another leader took, or past the four
    h = act ? (claim ? (slot + 1) & mask : q < 4u ? slot : (h + 4) & mask) : h;
  }
  return res;
}
// ---- spilled-collector blocks.  Tier-indexed Ctx members are read through selects, never a runtime
// array index: indexing an array member of the kernel's register-resident Ctx copy with a runtime
// value spills the whole Ctx to scratch (measured: 520-660 B/lane in every collector kernel).
template <typename T>
__device__ __forceinline__ T tier_sel(const T (&a)[NTIER], int t) {
  return t == 0 ? a[0] : t == 1 ? a[1] : t == 2 ? a[2] : a[3];
}
__device__ __forceinline__ uint32_t tier_words_d(int t) {
  return t == 0 ? tier_words(0) : t == 1 ? tier_words(1) : t == 2 ? tier_words(2) : tier_words(3);
}
__device__ __forceinline__ uint32_t* coll_block(const Ctx& c, uint32_t meta) {
  const int t = (int)((meta >> 4) & 3u);
  return tier_sel(c.spill, t) + (size_t)(meta >> 8) * tier_words_d(t);
}
__device__ inline uint32_t spill_alloc(const Ctx& c, int t) {
  const int32_t a = atomicSub(&c.spill_ctl[t].avail, 1);
  if (a > 0) return tier_sel(c.spill_avail, t)[a - 1];
  const uint32_t i = atomicAdd(&c.spill_ctl[t].bump, 1u);
  if (i >= tier_sel(c.spill_cap, t) || i >= (1u << 24)) { set_err(c, ERR_INTERVALS); return NONE; }
  return i;
}
__device__ inline void spill_free(const Ctx& c, uint32_t meta) {
  const int t = (int)((meta >> 4) & 3u);
  const uint32_t j = atomicAdd(&c.spill_ctl[t].freed, 1u);
  if (j < tier_sel(c.spill_cap, t)) tier_sel(c.spill_freed, t)[j] = meta >> 8;
}
// greatest i with iv[i].lo <= x, or -1 (TreeMap.floorEntry)
__device__ inline int coll_floor(const uint2* iv, uint32_t n, uint32_t x) {
  int lo = 0, hi = (int)n - 1, r = -1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (iv[mid].x <= x) { r = mid; lo = mid + 1; } else { hi = mid - 1; }
  }
  return r;
}
// SequenceIdCollector.contains (SequenceIdCollector.java:32-35)
__device__ inline bool coll_contains(const Ctx& c, const CollEnt* e, uint32_t x) {
  if (!e) return false;
  const uint32_t meta = e->meta, n = meta & 7u;
  if (n == 1) return e->lo <= x && x <= e->hi;
  if (n != COLL_SPILLED) return false;
  const uint32_t* blk = coll_block(c, meta);
  const uint2* iv = reinterpret_cast<const uint2*>(blk + 4);
  const int f = coll_floor(iv, blk[0], x);
  return f >= 0 && x <= iv[f].y;
}
// coll_contains on an entry already loaded (by value): the inline interval, else the spilled block
__device__ inline bool coll_contains_v(const Ctx& c, const CollEnt& e, uint32_t x) {
  const uint32_t n = e.meta & 7u;
  if (n == 1) return e.lo <= x && x <= e.hi;
  if (n != COLL_SPILLED) return false;
  const uint32_t* blk = coll_block(c, e.meta);
  const uint2* iv = reinterpret_cast<const uint2*>(blk + 4);
  const int f = coll_floor(iv, blk[0], x);
  return f >= 0 && x <= iv[f].y;
}
// "does receiver t's collector of `gossiper` hold seq?" for up to four receivers t at once (all owned):
// the first probe of each is loaded in one batch (the hash slot depends on the gossiper only), the
// rare continued probes and spilled blocks follow.  Bit q of the result: receiver tg[q] holds it
// (only bits set in `need` are examined).
__device__ inline uint32_t coll_known4(const Ctx& c, const uint32_t* tg, uint32_t need, uint32_t gossiper,
                                       uint32_t seq) {
  const uint32_t mask = c.hcap - 1, h = hash32(gossiper) & mask, key = gossiper + 1;
  CollEnt e[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if ((need >> q) & 1u) e[q] = c.coll[(size_t)(tg[q] - c.lo) * c.hcap + h];
  uint32_t known = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (!((need >> q) & 1u)) continue;
    if (e[q].key != key) {
      if (e[q].key == 0) continue;  // not in the table: nothing received from this gossiper
      const CollEnt* f = coll_find(c, tg[q], gossiper);
      if (!f) continue;
      e[q] = *f;
    }
    known |= coll_contains_v(c, e[q], seq) ? 1u << q : 0u;
  }
  return known;
}
// SequenceIdCollector.add (SequenceIdCollector.java:43-72).  `seg` (the viewer's segmentation flag)
// is raised when the collector ends up with more than c.seg_threshold intervals.  `pre`: the entry's
// current value when the caller holds it already (coll_ensure_v), so no load waits on it.
__device__ inline bool coll_add(const Ctx& c, CollEnt* e, uint32_t x, uint32_t* seg = nullptr,
                                const CollEnt* pre = nullptr) {
  if (!e) return true;
  uint32_t meta = pre ? pre->meta : e->meta;
  const uint32_t n0 = meta & 7u;
  if (n0 == 0) {
    e->lo = e->hi = x;
    e->meta = (meta & ~7u) | 1u;
    return true;
  }
  if (n0 == 1) {
    const uint32_t elo = pre ? pre->lo : e->lo, ehi = pre ? pre->hi : e->hi;
    if (elo <= x && x <= ehi) return false;
    if ((int64_t)x == (int64_t)ehi + 1) { e->hi = x; return true; }
    if ((int64_t)x + 1 == (int64_t)elo) { e->lo = x; return true; }
    const uint32_t lo0 = elo, hi0 = ehi;
    // a second disjoint interval: spill to the smallest tier
    const uint32_t i = spill_alloc(c, 0);
    if (i == NONE) return true;
    uint32_t* blk = c.spill[0] + (size_t)i * tier_words(0);
    uint2* iv = reinterpret_cast<uint2*>(blk + 4);
    if (x < lo0) { iv[0] = make_uint2(x, x); iv[1] = make_uint2(lo0, hi0); }
    else { iv[0] = make_uint2(lo0, hi0); iv[1] = make_uint2(x, x); }
    blk[0] = 2;
    e->meta = (meta & COLL_CLEARED) | COLL_SPILLED | (i << 8);
    if (seg && 2 > (uint32_t)c.seg_threshold) *seg = 1;
    return true;
  }
  uint32_t* blk = coll_block(c, meta);
  uint2* iv = reinterpret_cast<uint2*>(blk + 4);
  uint32_t n = blk[0];
  const int fl = coll_floor(iv, n, x);
  if (fl >= 0 && x <= iv[fl].y) return false;
  const int ce = fl + 1;  // first interval with lo > x
  const bool nf = fl >= 0 && (int64_t)x - 1 == (int64_t)iv[fl].y;
  const bool nc = ce < (int)n && (int64_t)x + 1 == (int64_t)iv[ce].x;
  if (nf && nc) {
    iv[fl].y = iv[ce].y;
    for (uint32_t i = (uint32_t)ce; i + 1 < n; ++i) iv[i] = iv[i + 1];
    n--;
  } else if (nf) {
    iv[fl].y = x;
  } else if (nc) {
    iv[ce].x = x;
  } else {
    const int t = (int)((meta >> 4) & 3u);
    if (n == (t == 0 ? tier_cap(0) : t == 1 ? tier_cap(1) : t == 2 ? tier_cap(2) : tier_cap(3))) {  // grow
      if (t + 1 == NTIER) { set_err(c, ERR_COLL_TOP); return true; }
      const uint32_t i = spill_alloc(c, t + 1);
      if (i == NONE) return true;
      uint32_t* nb = tier_sel(c.spill, t + 1) + (size_t)i * tier_words_d(t + 1);
      uint2* niv = reinterpret_cast<uint2*>(nb + 4);
      for (uint32_t k = 0; k < n; ++k) niv[k] = iv[k];
      spill_free(c, meta);
      meta = (meta & COLL_CLEARED) | COLL_SPILLED | ((uint32_t)(t + 1) << 4) | (i << 8);
      e->meta = meta;
      blk = nb;
      iv = niv;
    }
    for (uint32_t i = n; i > (uint32_t)ce; --i) iv[i] = iv[i - 1];
    iv[ce] = make_uint2(x, x);
    n++;
  }
  if (n == 1) {  // merged back into one interval: inline again
    e->lo = iv[0].x;
    e->hi = iv[0].y;
    spill_free(c, meta);
    e->meta = (meta & COLL_CLEARED) | 1u;
    return true;
  }
  blk[0] = n;
  if (seg && n > (uint32_t)c.seg_threshold) *seg = 1;
  return true;
}
// coll_add for a whole wave's run of adds to one collector (deliver_coop): the entry held in registers
// while it stays inline, else its intervals staged in LDS — the same sequence of adds, results and
// segmentation checks as coll_add one after another, without a dependent global round trip per add.
// On an inline value: 1 added, 0 held already, -1 a second disjoint interval (the caller stages it).
__device__ __forceinline__ int coll_add_inline(CollEnt& v, uint32_t x) {
  if ((v.meta & 7u) == 0u) {
    v.lo = v.hi = x;
    v.meta = (v.meta & ~7u) | 1u;
    return 1;
  }
  if (v.lo <= x && x <= v.hi) return 0;
  if ((int64_t)x == (int64_t)v.hi + 1) { v.hi = x; return 1; }
  if ((int64_t)x + 1 == (int64_t)v.lo) { v.lo = x; return 1; }
  return -1;
}
// on n sorted, disjoint, non-adjacent intervals in LDS (room for at least n + 1): 1 added, 0 held
__device__ inline int coll_add_lds(uint2* iv, uint32_t& n, uint32_t x, uint32_t* moved = nullptr) {
  int lo = 0, hi = (int)n - 1, fl = -1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (iv[mid].x <= x) { fl = mid; lo = mid + 1; } else { hi = mid - 1; }
  }
  if (fl >= 0 && x <= iv[fl].y) return 0;
  const int ce = fl + 1;
  const bool nf = fl >= 0 && (int64_t)x - 1 == (int64_t)iv[fl].y;
  const bool nc = ce < (int)n && (int64_t)x + 1 == (int64_t)iv[ce].x;
  if (nf && nc) {
    iv[fl].y = iv[ce].y;
    for (uint32_t i = (uint32_t)ce; i + 1 < n; ++i) iv[i] = iv[i + 1];
    if (moved) *moved += n - 1 - (uint32_t)ce;
    n--;
  } else if (nf) {
    iv[fl].y = x;
  } else if (nc) {
    iv[ce].x = x;
  } else {
    for (uint32_t i = n; i > (uint32_t)ce; --i) iv[i] = iv[i - 1];
    if (moved) *moved += n - (uint32_t)ce;
    iv[ce] = make_uint2(x, x);
    n++;
  }
  return 1;
}
// The same add made by the whole wave (every lane calls it with the same x; n is wave-uniform): the
// floor by binary search (every lane the same LDS reads), the intervals after the change moved 64 at
// a time.  One lane moving them one by one cost ~260 moves per add at config 3's churn (collectors of
// hundreds of intervals: 2.9 x 10^9 moves per delivery launch at N = 16,384).  Same result as
// coll_add_lds.  (wave_sync: this file's callers define it.)
template <typename Sync>
__device__ inline int coll_add_lds_wave(uint2* iv, uint32_t& n, uint32_t x, uint32_t lane, Sync wave_sync,
                                        uint32_t* moved = nullptr) {
  int lo = 0, hi = (int)n - 1, fl = -1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (iv[mid].x <= x) { fl = mid; lo = mid + 1; } else { hi = mid - 1; }
  }
  if (fl >= 0 && x <= iv[fl].y) return 0;
  const int ce = fl + 1;
  const bool nf = fl >= 0 && (int64_t)x - 1 == (int64_t)iv[fl].y;
  const bool nc = ce < (int)n && (int64_t)x + 1 == (int64_t)iv[ce].x;
  const uint32_t ce_hi = nc ? iv[ce].y : 0u;
  wave_sync();  // (every lane has read before any lane writes)
  if (nf && nc) {  // x joins its neighbours: [fl].y takes [ce].y, the intervals after ce move down one
    for (uint32_t b0 = (uint32_t)ce + 1; b0 < n; b0 += 64) {  // (ascending: a slot is read before it is overwritten)
      const uint32_t q = b0 + lane;
      uint2 v = make_uint2(0, 0);
      if (q < n) v = iv[q];
      wave_sync();
      if (q < n) iv[q - 1] = v;
      wave_sync();
    }
    if (lane == 0) iv[fl].y = ce_hi;
    if (moved) *moved += n - 1 - (uint32_t)ce;
    n--;
  } else if (nf) {
    if (lane == 0) iv[fl].y = x;
  } else if (nc) {
    if (lane == 0) iv[ce].x = x;
  } else {  // a new interval at ce: the intervals from ce on move up one, the top 64 first
    if ((int)n > ce) {
      for (int b0 = ce + (int)(((n - 1 - (uint32_t)ce) >> 6) << 6); b0 >= ce; b0 -= 64) {
        const uint32_t q = (uint32_t)b0 + lane;
        uint2 v = make_uint2(0, 0);
        if (q < n) v = iv[q];
        wave_sync();
        if (q < n) iv[q + 1] = v;
        wave_sync();
      }
    }
    if (lane == 0) iv[ce] = make_uint2(x, x);
    if (moved) *moved += n - (uint32_t)ce;
    n++;
  }
  wave_sync();
  return 1;
}
// coll_add made by the whole wave on a collector too big to stage in LDS (deliver_coop: thousands of
// intervals in a top-tier block).  The floor by a 64-way search (one gather of 64 pivots per step:
// 3 steps over 16,382 intervals, where coll_add makes 14 dependent loads), the intervals after the
// change moved 256 at a time (4 loads in flight per lane, then the 4 stores), where coll_add moves one
// interval per dependent round trip.  Same result as coll_add; the rare cases that change the entry's
// tier or inline value (a full block, a run back to one interval) are left to coll_add on lane 0.
// Every lane calls it with the same x; the return value is wave-uniform.
// (the 4 loads complete before the first store: one lane's store may land on another lane's next load)
#define COLL_WAVE_WAIT(v) \
  __asm__ volatile("" : "+v"(v[0].x), "+v"(v[0].y), "+v"(v[1].x), "+v"(v[1].y), "+v"(v[2].x), "+v"(v[2].y), \
                   "+v"(v[3].x), "+v"(v[3].y))
template <typename Sync>
__device__ inline int coll_add_wave(const Ctx& c, CollEnt* e, uint32_t x, uint32_t lane, Sync wave_sync,
                                    uint32_t* seg) {
  const uint32_t meta = rdlane(gload(&e->meta), 0);
  uint32_t* blk = (meta & 7u) == COLL_SPILLED ? coll_block(c, meta) : nullptr;
  const uint32_t n = blk ? rdlane(gload(blk), 0) : 0u;
  const int t = (int)((meta >> 4) & 3u);
  if (!blk || n <= 2u || n == tier_cap(t)) {  // one lane (coll_add), as before
    uint32_t r = 0;
    if (lane == 0) r = coll_add(c, e, x, seg) ? 1u : 0u;
    r = rdlane(r, 0);
    wave_sync();
    return (int)r;
  }
  uint2* iv = reinterpret_cast<uint2*>(blk + 4);
  // floor: the last interval with lo <= x, searched among [a, b) with 64 pivots a step
  int fl = -1;
  for (uint32_t a = 0, b = n; a < b;) {
    const uint32_t step = (b - a + 63u) >> 6;
    const uint32_t p = a + lane * step;
    const uint64_t le = __ballot(p < b && gload(&iv[p].x) <= x);
    if (!le) break;
    const uint32_t k = 63u - (uint32_t)__clzll((long long)le);
    fl = (int)(a + k * step);
    b = min(b, a + (k + 1u) * step);
    a = (uint32_t)fl + 1u;
  }
  const uint2 f = fl >= 0 ? gload(&iv[fl]) : make_uint2(0, 0);
  if (fl >= 0 && x <= f.y) return 0;
  const uint32_t ce = (uint32_t)(fl + 1);
  const uint2 cx = ce < n ? gload(&iv[ce]) : make_uint2(0, 0);
  const bool nf = fl >= 0 && (int64_t)x - 1 == (int64_t)f.y;
  const bool nc = ce < n && (int64_t)x + 1 == (int64_t)cx.x;
  uint32_t n1 = n;
  if (nf && nc) {  // x joins its neighbours: the intervals after ce move down one, ascending
    for (uint32_t b0 = ce + 1u; b0 < n; b0 += 256u) {
      uint2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t q = b0 + (uint32_t)u * 64u + lane;
        v[u] = q < n ? gload(&iv[q]) : make_uint2(0, 0);
      }
      COLL_WAVE_WAIT(v);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t q = b0 + (uint32_t)u * 64u + lane;
        if (q < n) iv[q - 1] = v[u];
      }
    }
    if (lane == 0) iv[fl].y = cx.y;
    n1 = n - 1;
  } else if (nf) {
    if (lane == 0) iv[fl].y = x;
  } else if (nc) {
    if (lane == 0) iv[ce].x = x;
  } else {  // a new interval at ce: the intervals from ce on move up one, the top 256 first
    for (int b0 = (int)n - 256; b0 + 256 > (int)ce; b0 -= 256) {
      uint2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = b0 + u * 64 + (int)lane;
        v[u] = q >= (int)ce ? gload(&iv[q]) : make_uint2(0, 0);
      }
      COLL_WAVE_WAIT(v);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = b0 + u * 64 + (int)lane;
        if (q >= (int)ce) iv[q + 1] = v[u];
      }
    }
    if (lane == 0) iv[ce] = make_uint2(x, x);
    n1 = n + 1;
  }
  if (lane == 0) {
    blk[0] = n1;
    if (seg && n1 > (uint32_t)c.seg_threshold) *seg = 1;
  }
  wave_sync();
  return 1;
}
// the staged intervals' home once the run is done (n after it, maxn the most it held): inline when one
// interval is left; else the entry's block if its tier holds maxn, or a block of the smallest tier that
// does (coll_add grows one tier at a time at each full insert: the same tier in the end; the old block
// is released).  Returns the block to copy the intervals into (header written), or null (inline, or the
// pool is dry: ERR_INTERVALS set by spill_alloc).  One lane.
__device__ inline uint32_t* coll_place(const Ctx& c, CollEnt* e, uint32_t meta, uint32_t n, uint32_t maxn,
                                       uint32_t lo0, uint32_t hi0) {
  const bool spilled = (meta & 7u) == COLL_SPILLED;
  if (n == 1) {  // (lo0, hi0): the one interval
    e->lo = lo0;
    e->hi = hi0;
    if (spilled) spill_free(c, meta);
    e->meta = (meta & COLL_CLEARED) | 1u;
    return nullptr;
  }
  const int t0 = spilled ? (int)((meta >> 4) & 3u) : 0;
  int t = t0;
  while (t + 1 < NTIER && tier_cap(t) < maxn) ++t;
  if (tier_cap(t) < maxn) { set_err(c, ERR_COLL_TOP); return nullptr; }
  uint32_t* blk;
  if (spilled && t == t0) {
    blk = coll_block(c, meta);
  } else {
    const uint32_t i = spill_alloc(c, t);
    if (i == NONE) return nullptr;
    if (spilled) spill_free(c, meta);
    meta = (meta & COLL_CLEARED) | COLL_SPILLED | ((uint32_t)t << 4) | (i << 8);
    e->meta = meta;
    blk = coll_block(c, meta);
  }
  blk[0] = n;
  return blk;
}
// number of intervals (checkGossipSegmentation's size())
__device__ inline uint32_t coll_size(const Ctx& c, const CollEnt* e) {
  const uint32_t n = e->meta & 7u;
  return n == COLL_SPILLED ? coll_block(c, e->meta)[0] : n;
}
// clear() / remove: no intervals, marked cleared (a GossipState may outlive its collector entries)
__device__ inline void coll_clear(const Ctx& c, CollEnt* e) {
  if ((e->meta & 7u) == COLL_SPILLED) spill_free(c, e->meta);
  e->meta = COLL_CLEARED;
}

// receipt bitmaps: receiver r (owned) accepted gossip (gossiper, seq) into its collector.  Sets the
// bit when the slot belongs to the gossip, else asks k_end_tick to hand the slot to it.
__device__ inline void receipt_mark(const Ctx& c, uint32_t r, uint32_t gossiper, uint32_t seq) {
  const uint64_t key = gkey(gossiper, seq);
  const uint32_t sl = gslot_of(key);
  const GSlot gs = c.gslot[sl];
  const uint64_t owner = gs.key;
  if (owner == key) {
    const uint32_t i = r - c.lo;
    atomicOr(&c.gbits[rbit_word(i, sl)], 1u << (sl & 31));
  } else if ((owner == 0ull || gs.tick + GSLOT_HOLD <= (uint32_t)c.T) &&
             // (an owner keeps its slot GSLOT_HOLD ticks: two live gossips on one slot would otherwise
             // take it from each other every tick, each claim clearing a bit in every receiver's row)
             c.gpend[sl] == 0ull &&  // (a plain read first: once claimed, the thousands of receivers of a
                                     // new gossip skip the contended compare-and-swap)
             atomicCAS(reinterpret_cast<unsigned long long*>(&c.gpend[sl]), 0ull, (unsigned long long)key) == 0ull) {
    const uint32_t par = (uint32_t)(c.T & 1);
    // at most one entry per slot; bit 31: the slot had an owner, whose bits the claim must clear (a
    // never-owned slot's bits are all zero: only an owned slot's gossip sets any)
    c.gclaim[par * GSLOTS + atomicAdd(&c.gclaim_cnt[par], 1u)] = sl | (owner ? 0x80000000u : 0u);
  }
}

// ------------------------------------------------------------------------------- events
// Appends from thousands of threads in one kernel (a timer storm removes a member at every viewer
// in one tick) go to SUBQ sub-queues picked by the wave, so no single counter serialises them;
// order is canonicalised on the host ((tick, viewer, phase, minor) sort).
constexpr uint32_t SUBQ = 16;
// sub-queue of an append for (viewer, subject): hashed, not by the appending wave — one lane may
// append thousands (a SYNC merge schedules a timer and emits an event per record it changes)
__device__ __forceinline__ uint32_t subq(uint32_t v, uint32_t s) { return ((v * 0x9E3779B1u) ^ (s * 0x85EBCA77u)) >> 28; }
__device__ inline void emit(const Ctx& c, uint32_t v, uint32_t s, uint32_t type, uint32_t phase, uint32_t minor,
                            uint32_t data = 0) {
  const uint32_t q = subq(v, s);
  uint32_t i = atomicAdd(&c.ev_cnt[q], 1u);
  if (i >= c.ev_cap) { set_err(c, ERR_EVENTS); return; }
  i += q * c.ev_cap;
  swim_event e;
  e.tick = c.T;
  e.viewer = v;
  e.subject = s;
  e.type = type;
  e.phase = phase;
  e.minor = minor;
  e.data = data;
  c.ev[i] = e;
}

// FailureDetectorImpl.onMemberEvent (:321-346) + GossipProtocolImpl.onMemberEvent (:238-261) for
// ADDED: the remote list append is O(1) and done now; the pingMembers insert is deferred to the end
// of the viewer's deliveries in this phase (apply_ins_batch), which applies its inserts in event order.
// Invariant the early exits of the delivery kernels rely on: ADDED is only published while a viewer
// processes received messages (gossip delivery, SYNC / SYNC_ACK merges), never by the timer or FD
// phases (publish_fd never admits ALIVE), so a phase without deliveries has no ops.
__device__ inline void on_added(const Ctx& c, uint32_t v, uint32_t s, uint32_t phase, uint32_t minor) {
  MemberDev& m = mem(c, v);
  remote_list(c, v)[m.remote_len] = s;
  m.remote_len++;
  // a viewer's ADDED events of one phase come from the one thread that owns it in that phase, so
  // its ops are in event order with no grouping pass
  InsOp op;
  op.s = s; op.phase = phase; op.minor = minor; op.next = NONE;
  const uint32_t rank = m.ins_rank;
  if (rank < INS_INLINE) {
    c.ins_inline[(size_t)(v - c.lo) * INS_INLINE + rank] = op;
  } else {
    uint32_t off, size;
    ins_block_of(rank - INS_INLINE, off, size);
    if (off == 0) {  // a new block: reserved whole, linked from the previous block's first op
      const uint32_t st = atomicAdd(c.ins_total, size);
      if (st + size > c.ins_cap) { set_err(c, ERR_INS); return; }
      if (rank == INS_INLINE) m.ins_head = st;
      else c.ins[m.ins_tail].next = st;
      m.ins_tail = st;  // (the current block's start)
    }
    c.ins[m.ins_tail + off] = op;
  }
  m.ins_rank = rank + 1;
}

// REMOVED: GossipProtocolImpl drops the member's SequenceIdCollector (:242); both lists drop the
// member before the viewer's next FD step (k_fd; they hold exactly the viewer's other `members`).
// REMOVED arises in the timer phase (DEAD is never gossiped or synced), where nothing reads the lists
// before the FD step, and in the FD step on a DEST_GONE ack, which removes the member from both lists
// itself (publish_fd).
// Safe under entry-parallel timer processing: only the (v, s) collector entry is written.
__device__ inline void on_removed(const Ctx& c, uint32_t v, uint32_t s) {
  CollEnt* e = coll_find(c, v, s);
  if (e) {
    coll_clear(c, e);
    c.clr_tick[v - c.lo] = (uint32_t)c.T;  // v's receipt bits predating this tick are void
    MemberDev& m = mem(c, v);
    m.clr_serial = m.gix_base + gsched(c, v).len;
  }
  c.compact_flag[v - c.lo] = 1u;
}

__device__ inline void publish_event(const Ctx& c, uint32_t v, uint32_t s, uint32_t type, uint32_t phase,
                                     uint32_t minor) {
  emit(c, v, s, type, phase, minor);
  if (type == SWIM_EV_ADDED) on_added(c, v, s, phase, minor);
  if (type == SWIM_EV_REMOVED) on_removed(c, v, s);
}

__device__ __forceinline__ uint32_t next_minor(const Ctx& c, uint32_t v, uint32_t phase, uint32_t s) {
  return phase == SWIM_PHASE_TIMERS ? s : mem(c, v).ev_minor++;
}

// ------------------------------------------------------------------------------- slab index
// GossipProtocolImpl.gossips.get(gossipId) (:206) is only needed when the member's collector of the
// gossiper was cleared (otherwise the collector proves the gossip new), so the index is built the
// first time a member needs it and kept up from then on.  It maps (gossiper, seq) to the gossip's
// slab serial (insertion number; slab[p] has serial gix_base + p): the sweep drops a prefix of the
// slab (infection periods grow along it), which only advances gix_base, and a slot whose serial fell
// below gix_base is free again.  Rebuilt from the slab when half its slots have been taken.
__device__ __forceinline__ uint32_t gix_hash(uint32_t g, uint32_t s) { return hash32(g * 0x9e3779b9u ^ s); }
__device__ __forceinline__ uint32_t* gix_of(const Ctx& c, uint32_t v) {
  return c.gix + (size_t)(v - c.lo) * (c.gix_mask + 1);
}
__device__ inline void gix_put(const Ctx& c, MemberDev& m, uint32_t len, uint32_t* ix, uint32_t g, uint32_t s, uint32_t serial) {
  const uint32_t mask = c.gix_mask;
  uint32_t h = gix_hash(g, s);
  for (uint32_t i = 0; i <= mask; ++i, ++h) {
    const uint32_t e = ix[h & mask];
    if (e == NONE || e - m.gix_base >= len) {  // empty, or a swept gossip's slot
      if (e == NONE) m.gix_used++;
      ix[h & mask] = serial;
      return;
    }
  }
  m.gix_valid = 0;  // unreachable at <= half load
}
// a gossip was appended at slab position gossip_len - 1
__device__ __forceinline__ void gix_note(const Ctx& c, MemberDev& m, uint32_t v, uint32_t g, uint32_t s) {
  if (!m.gix_valid) return;
  if (2 * m.gix_used >= c.gix_mask + 1) { m.gix_valid = 0; return; }
  const uint32_t len = gsched(c, v).len;
  gix_put(c, m, len, gix_of(c, v), g, s, m.gix_base + len - 1);
}
// a gossip was written at slab position pos (the whole-wave delivery, which appends several at once)
__device__ __forceinline__ void gix_note_at(const Ctx& c, MemberDev& m, uint32_t v, uint32_t g, uint32_t s, uint32_t pos,
                                            uint32_t len) {
  if (!m.gix_valid) return;
  if (2 * m.gix_used >= c.gix_mask + 1) { m.gix_valid = 0; return; }
  gix_put(c, m, len, gix_of(c, v), g, s, m.gix_base + pos);
}
// A GossipState can outlive its collector entry only if it predates a clear of the member's
// collectors: while every state in the slab was appended after the last clear (the sweep has dropped
// the older ones), a sequence id a cleared collector accepts has no state yet, as for any other
// collector, and the gossip lookup (and the index behind it) is not needed.
__device__ __forceinline__ bool pre_clear_states(const MemberDev& m) {
  return (int32_t)(m.clr_serial - m.gix_base) > 0;
}
// gix_put for many lanes at once (the whole-wave delivery): a free slot (empty, or a swept gossip's)
// is taken by compare-and-swap, so lanes racing for one slot each end in a slot of their own.  The
// slots taken differ from one-by-one inserts, the lookups' answers do not: a key sits in the first
// slot of its probe sequence that was free when it got there, and a slot never becomes empty again
// (swept slots stay non-empty until a rebuild).  Returns whether an empty slot was taken.
__device__ inline bool gix_put_atomic(uint32_t* ix, uint32_t mask, uint32_t base, uint32_t len, uint32_t g, uint32_t s,
                                      uint32_t serial) {
  uint32_t h = gix_hash(g, s);
  for (uint32_t i = 0; i <= mask; ++i, ++h) {
    uint32_t* slot = ix + (h & mask);
    uint32_t e = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (e == NONE || e - base >= len) {
      const uint32_t old = atomicCAS(slot, e, serial);
      if (old == e) return e == NONE;
      e = old;
    }
  }
  return false;  // (unreachable at <= half load)
}
// slab position of (g, s), or -1
__device__ inline int32_t gix_find(const Ctx& c, MemberDev& m, uint32_t v, const SlabRef& slab, uint32_t g,
                                   uint32_t s) {
  uint32_t* ix = gix_of(c, v);
  const uint32_t mask = c.gix_mask;
  const uint32_t len = gsched(c, v).len;
  if (!m.gix_valid) {
    for (uint32_t i = 0; i <= mask; ++i) ix[i] = NONE;
    m.gix_used = 0;
    m.gix_valid = 1;
    for (uint32_t p = 0; p < len; ++p) gix_put(c, m, len, ix, slab.H(p).gossiper, slab.H(p).seq, m.gix_base + p);
  }
  uint32_t h = gix_hash(g, s);
  for (uint32_t i = 0; i <= mask; ++i, ++h) {
    const uint32_t e = ix[h & mask];
    if (e == NONE) return -1;
    const uint32_t p = e - m.gix_base;
    if (p < len && slab.H(p).gossiper == g && slab.H(p).seq == s) return (int32_t)p;
  }
  return -1;
}

// ------------------------------------------------------------------------------- gossip origination
// spreadMembershipGossip (MembershipProtocolImpl.java:845-860) -> createAndPutGossip (GossipProtocolImpl.java:190-199)
// `why`: the call site (SWIM_ORIG_*), counted in swim_stats.gossips_by_reason
__device__ inline void spread_gossip(const Ctx& c, uint32_t v, uint32_t subject, uint32_t status, int32_t inc,
                                     uint32_t why) {
  MemberDev& m = mem(c, v);
  GossipSched& gs = gsched(c, v);
  if (gs.len >= c.gcap) { set_err(c, ERR_SLAB); return; }
  GossipDev g;
  g.gossiper = v;
  g.seq = (uint32_t)m.g_counter;
  g.subject = subject;
  g.status = status;
  g.inc = inc;
  g.inf_period = gs.period;
#pragma unroll
  for (int k = 0; k < GINF; ++k) g.inf[k] = NONE;
  if (gs.period > PER_MASK) set_err(c, ERR_INC);  // (2^28 gossip rounds)
  slab_of(c, v).put(gs.len, g);
  gs.len++;
  gix_note(c, m, v, g.gossiper, g.seq);
  m.g_counter++;
  CollEnt* e = coll_ensure(c, v, v);
  if (coll_add(c, e, g.seq, &c.seg_flag[v - c.lo])) receipt_mark(c, v, v, g.seq);
  stat_add(c, ST_GOSSIPS_CREATED, 1);
  stat_add(c, ST_ORIG0 + (int)why, 1);
}
// the SWIM_ORIG_* reason of a spreadMembershipGossipUnlessGossiped call (:836-843)
__device__ __forceinline__ uint32_t orig_of(int reason) { return reason == R_FD_EVENT ? SWIM_ORIG_FD : SWIM_ORIG_SYNC; }

// GossipProtocol.spread(Message) (GossipProtocolImpl.java:126-130): a user gossip, its payload in
// the subject field
__device__ inline void spread_user(const Ctx& c, uint32_t v, uint32_t payload) {
  MemberDev& m = mem(c, v);
  GossipSched& gs = gsched(c, v);
  if (gs.len >= c.gcap) { set_err(c, ERR_SLAB); return; }
  GossipDev g;
  g.gossiper = v;
  g.seq = (uint32_t)m.g_counter;
  g.subject = payload;
  g.status = SWIM_GOSSIP_USER;
  g.inc = 0;
  g.inf_period = gs.period;
#pragma unroll
  for (int k = 0; k < GINF; ++k) g.inf[k] = NONE;
  if (gs.period > PER_MASK) set_err(c, ERR_INC);  // (2^28 gossip rounds)
  slab_of(c, v).put(gs.len, g);
  gs.len++;
  gix_note(c, m, v, g.gossiper, g.seq);
  m.g_counter++;
  m.user_live++;
  CollEnt* e = coll_ensure(c, v, v);
  if (coll_add(c, e, g.seq, &c.seg_flag[v - c.lo])) receipt_mark(c, v, v, g.seq);
  stat_add(c, ST_GOSSIPS_CREATED, 1);
  stat_add(c, ST_ORIG0 + SWIM_ORIG_USER, 1);
}

// ------------------------------------------------------------------------------- timers
constexpr uint32_t WHEEL_FAILED = 0xfffffffeu;  // the page pool ran dry: releases the page's waiters
constexpr uint64_t WHEEL_EMPTY = ~0ull;  // an unwritten or consumed wheel slot (the pool starts all-empty)
__device__ __forceinline__ uint32_t b_of_deadline(const Ctx& c, uint64_t deadline) {
  return (uint32_t)(deadline & c.wheel_mask);
}
// a page from the recycled list, else a fresh one from the pool (WHEEL_FAILED when dry)
__device__ inline uint32_t wheel_page_alloc(const Ctx& c) {
  const int32_t a = atomicSub(&c.wheel_ctl->avail, 1);
  if (a > 0) return c.wheel_avail[a - 1];
  const uint32_t i = atomicAdd(&c.wheel_ctl->bump, 1u);
  return i < c.wheel_pages ? i : WHEEL_FAILED;
}

// scheduleSuspicionTimeoutTask (MembershipProtocolImpl.java:805-823)
__device__ __forceinline__ int32_t ceil_log2(uint32_t x) { return x ? 32 - __clz(x) : 0; }
__device__ inline void schedule_timer(const Ctx& c, uint32_t v, uint32_t s) {
  uint32_t* ap = aux_row(c, v) + s;
  const uint32_t a = *ap;
  if (a & A_HAS_TIMER) return;
  uint64_t ms = (uint64_t)c.suspicion_mult * (uint64_t)ceil_log2(mem(c, v).table_size) * (uint64_t)c.ping_interval;
  uint64_t deadline = c.T + ms / c.tick_ms;
  *ap = (a & 0xfu) | A_HAS_TIMER | ((uint32_t)(deadline & SWIM_DEADLINE_MASK) << 4);
  // queue of the viewer's 256-viewer block (fired by that block's k_fd workgroup)
  const uint32_t q = (size_t)b_of_deadline(c, deadline) * c.wheel_nq + ((v - c.lo) >> 8);
  const uint32_t i = atomicAdd(&c.wheel_cnt[q], 1u);
  const uint32_t pg = i >> c.wheel_pshift, slot = i & ((1u << c.wheel_pshift) - 1);
  if (pg >= c.wheel_ptmax) { set_err(c, ERR_WHEEL); return; }
  uint32_t* pt = c.wheel_pt + (size_t)q * c.wheel_ptmax + pg;
  // the writer of a page's first slot allocates it, the others wait for it; every lane of the wave
  // that reserved a slot here allocates before any lane waits, so a wave never waits on itself
  // (a lane that reserved an earlier slot elsewhere completed its own call before this one)
  const bool first = slot == 0;
  uint32_t pid = NONE;
  if (first) {
    pid = wheel_page_alloc(c);
    __atomic_store_n(pt, pid, __ATOMIC_RELAXED);
  }
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  if (!first)
    for (uint32_t it = 0; it < (1u << 22); ++it) {
      pid = __atomic_load_n(pt, __ATOMIC_RELAXED);
      if (pid != NONE) break;
      __builtin_amdgcn_s_sleep(1);
    }
  if (pid >= c.wheel_pages) { set_err(c, ERR_WHEEL); return; }  // pool dry (PG_FAILED) or timed out
  c.wheel[((size_t)pid << c.wheel_pshift) + slot] = ((uint64_t)v << 32) | s;
}

// ------------------------------------------------------------------------------- metadata fetch
// MetadataStoreImpl.fetchMetadata (:146-185) round trip + onMetadataRequest (:201-240), with the
// NetworkEmulator's arrival-time semantics: the request is lost or refused at its send and meets the
// subject's transport (stopped, inbound filter) when it arrives; the response likewise; the round
// trip must end before metadataTimeout (:160-165).  fetch_start returns true when the response is in
// within the calling phase (no delay on either leg: the caller applies the admission at its flush
// point); a delayed round trip is queued and completes in the FETCH phase of its arrival tick
// (k_fetch_due).  The oracle's fetch_start / fetch_stage1 / fetch_stage2 are the same steps.
__device__ inline void fq_push(const Ctx& c, uint32_t v, FetchEnt e) {
  const uint32_t p = (uint32_t)c.T & 1u;  // the queue written during tick T, read by tick T + 1
  const uint32_t slot = atomicAdd(&c.fq_cnt[p], 1u);
  if (slot >= c.fq_cap) { set_err(c, ERR_FETCHQ); return; }
  e.next = NONE;
  FetchEnt* q = c.fq + (size_t)p * c.fq_cap;
  q[slot] = e;
  const size_t li = (size_t)p * c.nl + (v - c.lo);
  if (c.fq_head[li] == NONE) c.fq_head[li] = slot;
  else q[c.fq_tail[li]].next = slot;
  c.fq_tail[li] = slot;
}
// the request arrives at d (now): 0 = the round trip failed, 1 = the response arrived too (no delay on
// it), 2 = the response is in flight (e.due = its arrival tick)
__device__ inline int fetch_stage1(const Ctx& c, uint32_t v, FetchEnt& e) {
  const uint32_t d = e.d, phase = e.info & 15u;
  if (!c.up[d] || !in_pass(c, d, v)) return 0;
  Ctx c0 = c;  // draws keyed by the issue tick
  c0.T = e.t0;
  if (out_fail(c0, d, v, v, SWIM_STREAM_FETCH_RESP, phase, e.f)) return 0;
  const uint32_t d2 = delay_ticks(c0, d, v, v, SWIM_STREAM_FETCH_RESP_DELAY, phase, e.f);
  if ((uint64_t)((uint32_t)c.T - e.t0 + d2) * c.tick_ms >= (uint64_t)c.metadata_timeout) return 0;
  e.ver = c.meta_ver[e.s];  // the metadata the response carries
  e.info = (e.info & 0xffu) | (2u << 8);
  e.due = (uint32_t)c.T + d2;
  if (d2 == 0) return c.up[v] && in_pass(c, v, d) ? 1 : 0;
  return 2;
}
// ticks from a fetch's send to its metadataTimeout (:160-165)
__device__ __forceinline__ uint32_t mt_ticks(const Ctx& c) { return (c.metadata_timeout + c.tick_ms - 1) / c.tick_ms; }
__device__ inline bool fetch_start(const Ctx& c, uint32_t v, uint32_t s, int32_t inc, int reason, uint32_t phase) {
  MemberDev& m = mem(c, v);
  const uint32_t f = m.fetch_ctr++;
  stat_add(c, ST_FETCHES, 1);
  const uint32_t lk1 = m.w_link1;  // a merge whose Monos are waited for (PAck)
  // the request goes to s's address; another member listening there does not answer (:209): the
  // Mono fails at metadataTimeout
  const uint32_t d = dst(c, s);
  const uint32_t to_tick = (uint32_t)c.T + mt_ticks(c);
  if (d != s) {
    if (lk1) m.w_ready = max(m.w_ready, to_tick);
    return false;
  }
  if (out_fail(c, v, d, v, SWIM_STREAM_FETCH_REQ, phase, f)) return false;  // fails at once
  const uint32_t d1 = delay_ticks(c, v, d, v, SWIM_STREAM_FETCH_REQ_DELAY, phase, f);
  if ((uint64_t)d1 * c.tick_ms >= (uint64_t)c.metadata_timeout) {
    if (lk1) m.w_ready = max(m.w_ready, to_tick);
    return false;
  }
  FetchEnt e;
  e.s = s; e.inc = inc; e.f = f; e.info = phase | ((uint32_t)reason << 4) | (1u << 8);
  e.d = d; e.ver = 0; e.t0 = (uint32_t)c.T; e.due = (uint32_t)c.T + d1; e.next = NONE;
  e.link = lk1 ? lk1 - 1 : NONE;
  if (d1 == 0) {
    const int r = fetch_stage1(c, v, e);
    if (r == 1) stat_add(c, ST_FETCH_OK, 1);
    if (r == 0 && lk1) m.w_ready = max(m.w_ready, to_tick);
    if (r != 2) return r == 1;
  }
  if (lk1) m.w_n++;
  fq_push(c, v, e);
  return false;
}

// ------------------------------------------------------------------------------- updateMembership
// MembershipProtocolImpl.updateMembership (:569-664).  Returns true when an ALIVE admission's
// metadata fetch succeeded: the caller applies it (apply_alive) at its flush point.
__device__ inline bool update_membership(const Ctx& c, uint32_t v, uint32_t s, uint32_t st1, int32_t inc1,
                                         int reason, uint32_t phase) {
  if (c.n_ns && !c.ns_rel[(size_t)c.ns[v] * c.n_ns + c.ns[s]]) return false;  // namespace filter (:575-586)
  MemberDev& m = mem(c, v);
  uint64_t cell = cell_get(c, v, s);
  const bool present = c_has(cell, B_IN_TABLE);
  const uint32_t st0 = c_status(cell);
  const int32_t inc0 = c_inc(cell);
  const bool r0_leaving = present && st0 == SWIM_LEAVING;
  if (!r0_leaving && !is_overrides(st1, inc1, present, st0, inc0)) return false;  // :593-602

  if (s == v) {  // onSelfMemberDetected (:686-708)
    int32_t cur = inc0 > inc1 ? inc0 : inc1;
    cell_put(c, v, s, c_with_record(cell, st0, cur + 1));
    spread_gossip(c, v, v, st0, cur + 1, SWIM_ORIG_REFUTE);
    return false;
  }
  if (dst(c, s) == v) return false;  // another member at the local address (:605-610)
  if (st1 == SWIM_LEAVING) {  // onLeavingDetected (:710-733)
    if (!present) m.table_size++;
    cell = c_with_record(cell | B_IN_TABLE, SWIM_LEAVING, inc1);
    cell_put(c, v, s, cell);
    if (present && (st0 == SWIM_ALIVE || (st0 == SWIM_SUSPECT && c_has(cell, B_ALIVE_EMITTED))))
      publish_event(c, v, s, SWIM_EV_LEAVING, phase, next_minor(c, v, phase, s));
    if (!present || st0 != SWIM_LEAVING) {
      schedule_timer(c, v, s);
      spread_gossip(c, v, s, SWIM_LEAVING, inc1, SWIM_ORIG_LEAVING);
      // onLeavingDetected returns the gossip's spread() Mono: a merge waits until it disseminated
      if (m.w_link1) m.w_gp = gsched(c, v).period + 1;
    }
    return false;
  }
  if (st1 == SWIM_DEAD) {  // onDeadMemberDetected (:740-767)
    cell &= ~B_HAS_TIMER;
    if (!c_has(cell, B_IN_MEMBERS)) { cell_put(c, v, s, cell); return false; }
    cell_put(c, v, s, 0);
    atomicSub(&m.table_size, 1u);  // atomic: timer buckets are processed entry-parallel
    atomicSub(&m.members_size, 1u);
    publish_event(c, v, s, SWIM_EV_REMOVED, phase, next_minor(c, v, phase, s));
    return false;
  }
  if (st1 == SWIM_SUSPECT) {  // :621-628
    if (!r0_leaving) {
      if (!present) m.table_size++;
      cell_put(c, v, s, c_with_record(cell | B_IN_TABLE, SWIM_SUSPECT, inc1));
    }
    schedule_timer(c, v, s);
    if (reason != R_GOSSIP && reason != R_INITIAL_SYNC) spread_gossip(c, v, s, SWIM_SUSPECT, inc1, orig_of(reason));
    return false;
  }
  // ALIVE (:630-660)
  if (r0_leaving) {  // onAliveAfterLeaving (:666-684)
    if (!c_has(cell, B_IN_MEMBERS)) { cell |= B_IN_MEMBERS; m.members_size++; }
    if (!c_has(cell, B_ALIVE_EMITTED)) {
      cell |= B_ALIVE_EMITTED;
      cell_put(c, v, s, cell);
      publish_event(c, v, s, SWIM_EV_ADDED, phase, next_minor(c, v, phase, s));
      publish_event(c, v, s, SWIM_EV_LEAVING, phase, next_minor(c, v, phase, s));
    } else {
      cell_put(c, v, s, cell);
    }
    return false;
  }
  if (!present || inc0 < inc1) return fetch_start(c, v, s, inc1, reason, phase);
  return false;
}

// A merged message's waits (PAck): collected between wait_begin and wait_end by the one thread that
// merges the message; wait_end makes a PAck when the message's Monos have not all completed by now
// (returns true: its SYNC_ACK, or the start0 group, waits).  Oracle: wait_begin / wait_end.
__device__ inline void wait_begin(const Ctx& c, uint32_t v) {
  MemberDev& m = mem(c, v);
  m.w_link1 = m.pack_seq + 1;
  m.w_n = m.w_ready = m.w_gp = 0;
}
__device__ inline bool wait_end(const Ctx& c, uint32_t v, uint32_t to, uint32_t flags) {
  MemberDev& m = mem(c, v);
  m.w_link1 = 0;
  if (m.w_n == 0 && m.w_gp == 0 && m.w_ready <= (uint32_t)c.T) return false;
  const uint32_t i = v - c.lo, k = c.pa_n[i];
  if (k >= c.pa_cap) {
    set_err(c, ERR_PACK);
    return true;
  }
  c.pa[(size_t)i * c.pa_cap + k] = PAck{to, flags, m.w_n, m.w_ready, m.w_gp, m.pack_seq};
  c.pa_n[i] = k + 1;
  m.pack_seq++;
  if (flags & PA_INIT) m.init_pend++;
  atomicOr(&c.mflag[i], MF_PACK);
  return true;
}
// the PAck of viewer v with sequence number seq (nullptr: none — a start0 group cancelled with its Flux)
__device__ inline PAck* pack_find(const Ctx& c, uint32_t v, uint32_t seq) {
  const uint32_t i = v - c.lo, k = min(c.pa_n[i], c.pa_cap);
  PAck* L = c.pa + (size_t)i * c.pa_cap;
  for (uint32_t j = 0; j < k; ++j)
    if (L[j].seq == seq) return L + j;
  return nullptr;
}

// doOnSuccess of the metadata fetch (:648-656) + onAliveMemberDetected (:769-795); ver = the
// subject's metadata version the response carried
__device__ inline void apply_alive(const Ctx& c, uint32_t v, uint32_t s, int32_t inc1, int reason, uint32_t phase,
                                   uint32_t ver) {
  MemberDev& m = mem(c, v);
  // cancelSuspicionTimeoutTask
  uint64_t cell = cell_get(c, v, s) & ~B_HAS_TIMER;
  // metadataStore.updateMetadata(member, metadata1) returns metadata0 (null when none is stored)
  bool same_meta = c_has(cell, B_HAS_METADATA);
  if (c.meta_seen) {
    uint32_t& seen = c.meta_seen[(size_t)(v - c.lo) * c.n + s];
    same_meta = same_meta && seen == ver;
    seen = ver;
  }
  cell |= B_HAS_METADATA;
  if (reason != R_GOSSIP && reason != R_INITIAL_SYNC) spread_gossip(c, v, s, SWIM_ALIVE, inc1, orig_of(reason));
  const bool exists = c_has(cell, B_IN_MEMBERS);
  if (!c_has(cell, B_IN_TABLE)) m.table_size++;
  if (!exists) m.members_size++;
  cell = c_with_record(cell | B_IN_TABLE | B_IN_MEMBERS, SWIM_ALIVE, inc1);
  if (!exists) cell |= B_ALIVE_EMITTED;
  cell_put(c, v, s, cell);
  if (!exists) publish_event(c, v, s, SWIM_EV_ADDED, phase, next_minor(c, v, phase, s));
  else if (!same_meta)  // !metadata1.equals(metadata0) (:780-781)
    publish_event(c, v, s, SWIM_EV_UPDATED, phase, next_minor(c, v, phase, s));
}

// a round trip answered within the phase: metadata1 is the subject's metadata now
__device__ inline void apply_alive(const Ctx& c, uint32_t v, uint32_t s, int32_t inc1, int reason, uint32_t phase) {
  apply_alive(c, v, s, inc1, reason, phase, c.meta_ver[s]);
}

// Collections.shuffle: for (i = size; i > 1; i--) swap(i-1, nextInt(i))
__device__ inline void shuffle_list(const Ctx& c, uint32_t v, uint32_t* list, uint32_t len, uint32_t stream) {
  for (uint32_t i = len; i > 1; --i) {
    uint32_t j = next_int(draw(c, v, stream, 0, i), i);
    uint32_t t = list[i - 1];
    list[i - 1] = list[j];
    list[j] = t;
  }
}

}  // namespace swimdev
