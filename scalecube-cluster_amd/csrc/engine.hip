// engine.hip — host orchestration and C ABI (include/swim.h) of libswimgpu.so.
//
// One swim_engine owns all device memory of one simulated cluster on the current HIP device and
// advances it tick by tick with the kernel sequence of swim_kernels.h on one HIP stream.  No host
// synchronisation happens inside a tick; the host syncs once per swim_step_ticks call (and every
// kDrainEvery ticks) to move events to the host buffer and to check the capacity-error word.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "swim_phases.h"

using namespace swimdev;

namespace {

constexpr uint32_t kDrainEvery = 256;
constexpr uint32_t kClassifyGrid = 2048;  // grid-stride over (message, chunk) work units
constexpr uint32_t kApplyGrid = 256;      // grid-stride over receivers

uint32_t gcd_u(uint32_t a, uint32_t b) {
  while (b) { uint32_t t = a % b; a = b; b = t; }
  return a;
}
uint32_t next_pow2(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
int32_t host_ceil_log2(int32_t num) {
  uint32_t u = (uint32_t)num;
  int32_t r = 0;
  while (u) { u >>= 1; r++; }
  return r;
}

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, sizeof(T) * (count ? count : 1));
}

}  // namespace

struct swim_engine {
  swim_config cfg{};
  int32_t device = 0;
  uint32_t n = 0, tick_ms = 0, P = 0, G = 0, S = 0;
  uint64_t T = 0;
  hipStream_t stream = nullptr;
  Ctx c{};
  Bufs b{};
  Counters* k = nullptr;
  CollDev* kat_coll = nullptr;
  // host mirrors
  std::vector<uint8_t> g_residue;  // gossip timer residues mod G in use
  std::vector<uint32_t> seeds;
  std::vector<uint8_t> is_seed_h;
  std::vector<LinkDev> links_h;
  uint32_t links_dev_cap = 0;
  bool joins_pending = false;
  std::vector<swim_event> events;
  uint64_t host_ticks = 0, host_events = 0;
  uint32_t err_seen = 0;
  std::vector<void*> allocs;
  // swim_profile_*: HIP events around every k_sync_merge launch on `stream`
  bool prof = false;
  std::vector<hipEvent_t> prof_ev;
  uint32_t prof_used = 0;
  double prof_ms = 0;
  uint64_t prof_launches = 0;
  unsigned long long prof_base_msgs = 0, prof_base_recs = 0;

  ~swim_engine() {
    if (stream) hipStreamSynchronize(stream);
    for (hipEvent_t ev : prof_ev) hipEventDestroy(ev);
    for (void* p : allocs) hipFree(p);
    if (stream) hipStreamDestroy(stream);
  }
  template <typename T>
  bool alloc(T** p, size_t count) {
    if (dalloc(p, count) != hipSuccess) return false;
    allocs.push_back((void*)*p);
    return true;
  }
};

static int32_t hip_status() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    std::fprintf(stderr, "libswimgpu: HIP error %s\n", hipGetErrorString(e));
    return SWIM_EDEVICE;
  }
  return SWIM_OK;
}

static uint32_t grid_for(uint32_t n, uint32_t block) { return std::max(1u, (n + block - 1) / block); }

// device counters are replicated ST_REPL times; sum them
static int32_t read_stats(swim_engine* e, unsigned long long* st) {
  std::vector<unsigned long long> rep((size_t)ST_COUNT * ST_REPL);
  if (hipMemcpy(rep.data(), e->c.stats, sizeof(unsigned long long) * rep.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return SWIM_EDEVICE;
  for (int s = 0; s < ST_COUNT; ++s) {
    st[s] = 0;
    for (int r = 0; r < ST_REPL; ++r) st[s] += rep[(size_t)s * ST_REPL + r];
  }
  return SWIM_OK;
}

static void prof_flush(swim_engine* e) {
  for (uint32_t i = 0; i < e->prof_used; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e->prof_ev[2 * i], e->prof_ev[2 * i + 1]) == hipSuccess) e->prof_ms += ms;
  }
  e->prof_launches += e->prof_used;
  e->prof_used = 0;
}

static void launch_classify(swim_engine* e, int d2) {
  const bool p = e->prof && 2 * (e->prof_used + 1) <= e->prof_ev.size();
  if (p) hipEventRecord(e->prof_ev[2 * e->prof_used], e->stream);
  k_sync_classify<<<kClassifyGrid, CLS_BLOCK, 0, e->stream>>>(e->c, e->b, d2);
  if (p) {
    hipEventRecord(e->prof_ev[2 * e->prof_used + 1], e->stream);
    e->prof_used++;
  }
}

static int32_t sync_and_collect(swim_engine* e) {
  if (hipStreamSynchronize(e->stream) != hipSuccess) return hip_status() ? SWIM_EDEVICE : SWIM_EDEVICE;
  uint32_t cnt = 0, err = 0;
  if (hipMemcpy(&cnt, e->c.ev_cnt, 4, hipMemcpyDeviceToHost) != hipSuccess) return SWIM_EDEVICE;
  if (hipMemcpy(&err, e->c.err, 4, hipMemcpyDeviceToHost) != hipSuccess) return SWIM_EDEVICE;
  cnt = std::min(cnt, e->c.ev_cap);
  if (cnt) {
    size_t old = e->events.size();
    e->events.resize(old + cnt);
    if (hipMemcpy(e->events.data() + old, e->c.ev, sizeof(swim_event) * cnt, hipMemcpyDeviceToHost) != hipSuccess)
      return SWIM_EDEVICE;
    e->host_events += cnt;
    uint32_t zero = 0;
    if (hipMemcpy(e->c.ev_cnt, &zero, 4, hipMemcpyHostToDevice) != hipSuccess) return SWIM_EDEVICE;
  }
  e->err_seen |= err;
  if (e->prof) prof_flush(e);
  return err ? SWIM_ECAPACITY : SWIM_OK;
}

// deferred pingMembers inserts of the phase's ADDED events (Ctx points at that phase's counters)
static void run_ins_pipeline(swim_engine* e, const Ctx& c) {
  k_ins_prep<<<1, 1024, 0, e->stream>>>(c, e->b);
  k_ins_apply<<<512, 256, 0, e->stream>>>(c, e->b);
}

// One tick = 15 kernels (21 on gossip ticks) on one stream; no host synchronisation.
static void run_tick(swim_engine* e) {
  e->T += 1;
  e->host_ticks += 1;
  Ctx& c = e->c;
  Bufs& b = e->b;
  c.T = e->T;
  hipStream_t s = e->stream;
  const uint32_t n = e->n;
  const uint32_t gm = grid_for(n, 256);
  if (e->joins_pending) {
    k_start_joins<<<gm, 256, 0, s>>>(c);
    e->joins_pending = false;
  }
  // ---- A: suspicion timeouts
  const uint32_t bucket = (uint32_t)(e->T & c.wheel_mask);
  k_timers<<<256, 256, 0, s>>>(c, bucket);
  k_compact<<<256, 256, 0, s>>>(c, e->k, bucket);
  // ---- B: failure detector
  k_fd<<<gm, 256, 0, s>>>(c);
  // ---- C: gossip round
  if (e->g_residue[e->T % e->G]) {
    if (c.seg_threshold < KIV) k_gossip_seg<<<gm, 256, 0, s>>>(c);
    k_gossip_emit<<<gm, 256, 0, s>>>(c, b);
    k_alloc<<<64, 256, 0, s>>>(b.msg_recv, &e->k->msg_recv_cnt, b.msg_cnt, b.msg_start, &e->k->msg_cursor);
    k_scatter_msgs<<<512, 256, 0, s>>>(b);
    k_gossip_deliver<<<gm, 256, 0, s>>>(c, b);
    run_ins_pipeline(e, c);
  }
  // ---- D: SYNC / SYNC_ACK (list inserts use the second set of counters)
  Ctx cd = c;
  cd.ins_total = &e->k->ins_total2;
  cd.ins_list_cnt = &e->k->ins_list_cnt2;
  k_sync_collect<<<gm, 256, 0, s>>>(cd, b);
  for (int d2 = 0; d2 < 2; ++d2) {
    k_sync_prep<<<1, 1024, 0, s>>>(cd, b, d2);
    launch_classify(e, d2);
    k_sync_apply<<<kApplyGrid, APPLY_BLOCK, 0, s>>>(cd, b, d2);
  }
  run_ins_pipeline(e, cd);
  // ---- end of tick (also zeroes the per-tick counters)
  k_end_tick<<<gm, 256, 0, s>>>(c, e->k);
}

static int32_t upload_links(swim_engine* e) {
  auto& L = e->links_h;
  std::sort(L.begin(), L.end(), [](const LinkDev& x, const LinkDev& y) { return x.a < y.a || (x.a == y.a && x.b < y.b); });
  if (L.size() > e->links_dev_cap) {
    if (hipSetDevice(e->device) != hipSuccess) return SWIM_EDEVICE;
    uint32_t cap = next_pow2((uint32_t)L.size());
    LinkDev* p = nullptr;
    if (!e->alloc(&p, cap)) return SWIM_ENOMEM;
    e->c.links = p;
    e->links_dev_cap = cap;
  }
  if (!L.empty() && hipMemcpy(e->c.links, L.data(), sizeof(LinkDev) * L.size(), hipMemcpyHostToDevice) != hipSuccess)
    return SWIM_EDEVICE;
  e->c.n_links = (uint32_t)L.size();
  return SWIM_OK;
}

static LinkDev* find_link_h(swim_engine* e, uint32_t a, uint32_t b, bool create) {
  for (auto& L : e->links_h)
    if (L.a == a && L.b == b) return &L;
  if (!create) return nullptr;
  e->links_h.push_back(LinkDev{a, b, -1, -1});
  return &e->links_h.back();
}

static void prune_links(swim_engine* e) {
  auto& L = e->links_h;
  L.erase(std::remove_if(L.begin(), L.end(), [](const LinkDev& x) { return x.out_loss < 0 && x.in_pass < 0; }), L.end());
}

template <typename F>
static int32_t member_field_write(swim_engine* e, uint32_t m, size_t offset, const F& val) {
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  char* base = reinterpret_cast<char*>(e->c.mem + m) + offset;
  return hipMemcpy(base, &val, sizeof(F), hipMemcpyHostToDevice) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
}

static int32_t read_member_dev(swim_engine* e, uint32_t m, MemberDev* out) {
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return hipMemcpy(out, e->c.mem + m, sizeof(MemberDev), hipMemcpyDeviceToHost) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
}

// leaveCluster (MembershipProtocolImpl.java:233-242) on the device: LEAVING inc+1, spread gossip
__global__ void k_leave(Ctx c, uint32_t v, int32_t stop_after) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  MemberDev& m = c.mem[v];
  uint64_t* cp = row(c, v) + v;
  int32_t inc = c_inc(*cp) + 1;
  *cp = c_with_record(*cp, SWIM_LEAVING, inc);
  spread_gossip(c, v, v, SWIM_LEAVING, inc);
  if (stop_after) {
    m.leave_pending = 1;
    m.leave_gossiper = v;
    m.leave_seq = m.g_counter - 1;
  }
}

extern "C" {

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
  if (preset == 1) {  // defaultWanConfig
    c->ping_timeout = 3000;
    c->ping_interval = 5000;
    c->gossip_fanout = 4;
    c->suspicion_mult = 6;
    c->sync_interval = 60000;
    c->metadata_timeout = 10000;
  } else if (preset == 2) {  // defaultLocalConfig
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

int32_t swim_ceil_log2(int32_t num) { return host_ceil_log2(num); }
int32_t swim_gossip_periods_to_spread(int32_t repeat_mult, int32_t cluster_size) {
  return repeat_mult * host_ceil_log2(cluster_size);
}
int32_t swim_gossip_periods_to_sweep(int32_t repeat_mult, int32_t cluster_size) {
  return 2 * (swim_gossip_periods_to_spread(repeat_mult, cluster_size) + 1);
}
int64_t swim_suspicion_timeout(int32_t suspicion_mult, int32_t cluster_size, int64_t ping_interval) {
  return (int64_t)(suspicion_mult * host_ceil_log2(cluster_size)) * ping_interval;
}

int32_t swim_create(const swim_config* cfg, uint32_t capacity, uint32_t n_initial, uint64_t seed, swim_engine** out) {
  if (!cfg || !out || capacity < 2 || n_initial > capacity || capacity > (1u << 24)) return SWIM_EINVAL;
  const swim_config& cf = *cfg;
  if (cf.ping_interval <= 0 || cf.ping_timeout <= 0 || cf.ping_timeout >= cf.ping_interval || cf.gossip_interval <= 0 ||
      cf.sync_interval <= 0 || cf.sync_timeout <= 0 || cf.metadata_timeout <= 0 || cf.suspicion_mult <= 0 ||
      cf.gossip_fanout <= 0 || cf.gossip_fanout > 16 || cf.ping_req_members > 16 || cf.gossip_repeat_mult <= 0)
    return SWIM_EINVAL;
  uint32_t tick = (uint32_t)cf.tick_ms;
  if (tick == 0) {
    tick = gcd_u((uint32_t)cf.ping_interval, (uint32_t)cf.ping_timeout);
    tick = gcd_u(tick, (uint32_t)cf.gossip_interval);
    tick = gcd_u(tick, (uint32_t)cf.sync_interval);
    tick = gcd_u(tick, (uint32_t)cf.sync_timeout);
  }
  if (cf.ping_interval % tick || cf.ping_timeout % tick || cf.gossip_interval % tick || cf.sync_interval % tick ||
      cf.sync_timeout % tick)
    return SWIM_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return SWIM_EDEVICE;
  if (cf.device < 0 || cf.device >= ndev) return SWIM_EINVAL;
  if (hipSetDevice(cf.device) != hipSuccess) return SWIM_EDEVICE;

  swim_engine* e = new (std::nothrow) swim_engine();
  if (!e) return SWIM_ENOMEM;
  e->cfg = cf;
  e->device = cf.device;
  e->n = capacity;
  e->tick_ms = tick;
  e->P = (uint32_t)cf.ping_interval / tick;
  e->G = (uint32_t)cf.gossip_interval / tick;
  e->S = (uint32_t)cf.sync_interval / tick;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) { delete e; return SWIM_EDEVICE; }

  Ctx& c = e->c;
  Bufs& b = e->b;
  const uint32_t n = capacity;
  c.n = n;
  c.gcap = cf.gossip_capacity ? cf.gossip_capacity : 1024;
  c.hcap = next_pow2(cf.collector_capacity ? cf.collector_capacity : 1024);
  c.P = e->P;
  c.to_ticks = (uint32_t)cf.ping_timeout / tick;
  c.relay_ticks = e->P - c.to_ticks;
  c.G = e->G;
  c.S = e->S;
  c.sync_to_ticks = (uint32_t)cf.sync_timeout / tick;
  c.tick_ms = tick;
  c.ping_interval = cf.ping_interval;
  c.suspicion_mult = cf.suspicion_mult;
  c.repeat_mult = cf.gossip_repeat_mult;
  c.fanout = cf.gossip_fanout;
  c.ping_req_members = cf.ping_req_members;
  c.seg_threshold = cf.gossip_segmentation_threshold;
  c.record_fd = cf.record_fd_events;
  c.key0 = (uint32_t)seed;
  c.key1 = (uint32_t)(seed >> 32);
  const uint64_t max_timer = (uint64_t)cf.suspicion_mult * (uint64_t)host_ceil_log2((int32_t)n) * e->P;
  c.wheel_mask = next_pow2((uint32_t)max_timer + 2) - 1;
  c.wheel_cap = std::max<uint32_t>(4096, 2 * n);
  c.ev_cap = cf.event_capacity ? cf.event_capacity : (1u << 22);
  c.ins_cap = std::max<uint32_t>(1u << 16, 4 * n);
  b.msg_cap = (uint32_t)std::min<uint64_t>(1ull << 28, std::max<uint64_t>(1ull << 20, 256ull * n));
  b.req_cap = std::max<uint32_t>(1u << 12, 4 * n);
  b.snap_cap = 64;
  b.chunks = (n + SYNC_CHUNK - 1) / SYNC_CHUNK;
  b.pool_cap = std::max<uint32_t>(1u << 22, 16 * n);

  const size_t nn = (size_t)n * n;
  bool ok = e->alloc(&c.cells, nn) && e->alloc(&c.mem, n) && e->alloc(&c.ping, nn) && e->alloc(&c.remote, nn) &&
            e->alloc(&c.slab, (size_t)n * c.gcap) && e->alloc(&c.coll, (size_t)n * c.hcap) &&
            e->alloc(&c.fd_sync, (size_t)n * FD_SYNC_MAX) && e->alloc(&c.wheel, (size_t)(c.wheel_mask + 1) * c.wheel_cap) &&
            e->alloc(&c.wheel_cnt, c.wheel_mask + 1) && e->alloc(&c.ev, c.ev_cap) && e->alloc(&c.ev_cnt, 1) &&
            e->alloc(&c.default_loss, n) && e->alloc(&c.default_inbound, n) && e->alloc(&c.group, n) &&
            e->alloc(&c.links, 1) && e->alloc(&c.is_seed, n) && e->alloc(&c.seeds, n) && e->alloc(&c.ins, c.ins_cap) &&
            e->alloc(&c.ins_cnt, n) && e->alloc(&c.ins_list, n) && e->alloc(&c.compact_flag, n) &&
            e->alloc(&c.compact_list, n) && e->alloc(&c.stats, (size_t)ST_COUNT * ST_REPL) && e->alloc(&c.err, 1) &&
            e->alloc(&e->k, 1) && e->alloc(&b.msgs, b.msg_cap) && e->alloc(&b.msgs_out, b.msg_cap) &&
            e->alloc(&b.msg_cnt, n) && e->alloc(&b.msg_start, n) && e->alloc(&b.msg_recv, n) &&
            e->alloc(&b.reqs, b.req_cap) && e->alloc(&b.reqs_out, b.req_cap) && e->alloc(&b.req_cnt, n) &&
            e->alloc(&b.req_start, n) && e->alloc(&b.req_recv, n) && e->alloc(&b.acks, b.req_cap) &&
            e->alloc(&b.acks_out, b.req_cap) && e->alloc(&b.ack_cnt, n) && e->alloc(&b.ack_start, n) &&
            e->alloc(&b.ack_recv, n) && e->alloc(&b.ins_out, c.ins_cap) && e->alloc(&b.ins_start, n) &&
            e->alloc(&b.snap, (size_t)b.snap_cap * n) && e->alloc(&b.snap_idx, n) && e->alloc(&b.snap_list, b.snap_cap) &&
            e->alloc(&b.snap_cnt, 1) && e->alloc(&b.item_chunk, (size_t)b.req_cap * b.chunks) &&
            e->alloc(&b.item_total, b.req_cap) &&
            e->alloc(&b.pool, b.pool_cap) && e->alloc(&b.pend, (size_t)kApplyGrid * n) && e->alloc(&e->kat_coll, 1);
  if (!ok) { delete e; return SWIM_ENOMEM; }
  c.links = e->c.links;
  e->links_dev_cap = 1;
  c.ins_total = &e->k->ins_total;
  c.ins_list_cnt = &e->k->ins_list_cnt;
  c.compact_cnt = &e->k->compact_cnt;
  b.k = e->k;
  hipStream_t s = e->stream;
  hipMemsetAsync(c.coll, 0, sizeof(CollDev) * (size_t)n * c.hcap, s);
  hipMemsetAsync(c.wheel_cnt, 0, sizeof(uint32_t) * (c.wheel_mask + 1), s);
  hipMemsetAsync(c.ev_cnt, 0, 4, s);
  hipMemsetAsync(c.default_loss, 0, n, s);
  hipMemsetAsync(c.default_inbound, 1, n, s);
  hipMemsetAsync(c.group, 0, 2 * (size_t)n, s);
  hipMemsetAsync(c.is_seed, 0, n, s);
  hipMemsetAsync(c.ins_cnt, 0, 4 * (size_t)n, s);
  hipMemsetAsync(c.compact_flag, 0, 4 * (size_t)n, s);
  hipMemsetAsync(c.stats, 0, 8 * (size_t)ST_COUNT * ST_REPL, s);
  hipMemsetAsync(c.err, 0, 4, s);
  hipMemsetAsync(e->k, 0, sizeof(Counters), s);
  hipMemsetAsync(b.msg_cnt, 0, 4 * (size_t)n, s);
  hipMemsetAsync(b.req_cnt, 0, 4 * (size_t)n, s);
  hipMemsetAsync(b.ack_cnt, 0, 4 * (size_t)n, s);
  hipMemsetAsync(b.snap_idx, 0xff, 4 * (size_t)n, s);
  hipMemsetAsync(b.snap_cnt, 0, 4, s);
  c.T = 0;
  k_init_rows<<<std::min<uint32_t>(n, 65535), 256, 0, s>>>(c, n_initial);
  k_init_members<<<grid_for(n, 64), 64, 0, s>>>(c, n_initial, cf.sync_stagger);
  if (hipStreamSynchronize(s) != hipSuccess || hip_status() != SWIM_OK) { delete e; return SWIM_EDEVICE; }
  e->g_residue.assign(e->G, 0);
  e->g_residue[0] = 1;
  e->is_seed_h.assign(n, 0);
  *out = e;
  return SWIM_OK;
}

int32_t swim_destroy(swim_engine* e) {
  delete e;
  return SWIM_OK;
}

int32_t swim_step_ticks(swim_engine* e, uint32_t ticks) {
  if (!e) return SWIM_EINVAL;
  if (hipSetDevice(e->device) != hipSuccess) return SWIM_EDEVICE;
  int32_t rc = SWIM_OK;
  for (uint32_t i = 0; i < ticks; ++i) {
    run_tick(e);
    if ((i + 1) % kDrainEvery == 0) {
      int32_t r = sync_and_collect(e);
      if (r == SWIM_EDEVICE) return r;
    }
  }
  if (hip_status() != SWIM_OK) return SWIM_EDEVICE;
  rc = sync_and_collect(e);
  return rc;
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

int32_t swim_set_seeds(swim_engine* e, const uint32_t* seeds, uint32_t n_seeds) {
  if (!e || (n_seeds && !seeds)) return SWIM_EINVAL;
  std::vector<uint32_t> s;
  for (uint32_t i = 0; i < n_seeds; ++i) {
    if (seeds[i] >= e->n) return SWIM_EINVAL;
    if (std::find(s.begin(), s.end(), seeds[i]) == s.end()) s.push_back(seeds[i]);
  }
  e->seeds = s;
  std::fill(e->is_seed_h.begin(), e->is_seed_h.end(), 0);
  for (uint32_t x : s) e->is_seed_h[x] = 1;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  if (!s.empty() && hipMemcpy(e->c.seeds, s.data(), 4 * s.size(), hipMemcpyHostToDevice) != hipSuccess) return SWIM_EDEVICE;
  if (hipMemcpy(e->c.is_seed, e->is_seed_h.data(), e->n, hipMemcpyHostToDevice) != hipSuccess) return SWIM_EDEVICE;
  e->c.n_seeds = (uint32_t)s.size();
  return SWIM_OK;
}

int32_t swim_kill(swim_engine* e, uint32_t m) {
  if (!e || m >= e->n) return SWIM_EINVAL;
  MemberDev md;
  if (read_member_dev(e, m, &md) != SWIM_OK) return SWIM_EDEVICE;
  if (!md.up) return SWIM_ESTATE;
  md.up = 0;
  md.leave_pending = 0;
  return hipMemcpy(e->c.mem + m, &md, sizeof(MemberDev), hipMemcpyHostToDevice) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
}

int32_t swim_leave(swim_engine* e, uint32_t m, int32_t stop_after) {
  if (!e || m >= e->n) return SWIM_EINVAL;
  MemberDev md;
  if (read_member_dev(e, m, &md) != SWIM_OK) return SWIM_EDEVICE;
  if (!md.up) return SWIM_ESTATE;
  e->c.T = e->T;
  k_leave<<<1, 64, 0, e->stream>>>(e->c, m, stop_after);
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return hip_status();
}

int32_t swim_join(swim_engine* e, uint32_t m) {
  if (!e || m >= e->n) return SWIM_EINVAL;
  MemberDev md;
  if (read_member_dev(e, m, &md) != SWIM_OK) return SWIM_EDEVICE;
  if (md.joined || md.up || md.join_pending) return SWIM_ESTATE;
  md.join_pending = 1;
  if (hipMemcpy(e->c.mem + m, &md, sizeof(MemberDev), hipMemcpyHostToDevice) != hipSuccess) return SWIM_EDEVICE;
  e->joins_pending = true;
  e->g_residue[(e->T + 1) % e->G] = 1;  // the joiner's gossip timer phase
  return SWIM_OK;
}

int32_t swim_set_default_loss(swim_engine* e, uint32_t m, int32_t pct) {
  if (!e || pct < 0 || pct > 100) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  if (m == 0xffffffffu) return hipMemset(e->c.default_loss, pct, e->n) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
  if (m >= e->n) return SWIM_EINVAL;
  uint8_t v = (uint8_t)pct;
  return hipMemcpy(e->c.default_loss + m, &v, 1, hipMemcpyHostToDevice) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
}

int32_t swim_set_link_loss(swim_engine* e, uint32_t src, uint32_t dst, int32_t pct) {
  if (!e || src >= e->n || dst >= e->n || pct > 100) return SWIM_EINVAL;
  if (pct < 0) {
    LinkDev* L = find_link_h(e, src, dst, false);
    if (L) L->out_loss = -1;
  } else {
    find_link_h(e, src, dst, true)->out_loss = pct;
  }
  prune_links(e);
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return upload_links(e);
}

int32_t swim_set_link_inbound(swim_engine* e, uint32_t dst, uint32_t src, int32_t pass) {
  if (!e || src >= e->n || dst >= e->n) return SWIM_EINVAL;
  if (pass < 0) {
    LinkDev* L = find_link_h(e, dst, src, false);
    if (L) L->in_pass = -1;
  } else {
    find_link_h(e, dst, src, true)->in_pass = pass ? 1 : 0;
  }
  prune_links(e);
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return upload_links(e);
}

int32_t swim_set_default_inbound(swim_engine* e, uint32_t m, int32_t pass) {
  if (!e) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  if (m == 0xffffffffu) return hipMemset(e->c.default_inbound, pass ? 1 : 0, e->n) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
  if (m >= e->n) return SWIM_EINVAL;
  uint8_t v = pass ? 1 : 0;
  return hipMemcpy(e->c.default_inbound + m, &v, 1, hipMemcpyHostToDevice) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
}

int32_t swim_set_partition(swim_engine* e, const uint16_t* g) {
  if (!e) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  if (!g) { e->c.partition = 0; return SWIM_OK; }
  if (hipMemcpy(e->c.group, g, 2 * (size_t)e->n, hipMemcpyHostToDevice) != hipSuccess) return SWIM_EDEVICE;
  e->c.partition = 1;
  return SWIM_OK;
}

int32_t swim_read_view(swim_engine* e, uint32_t v, uint64_t* out) {
  if (!e || v >= e->n || !out) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return hipMemcpy(out, e->c.cells + (size_t)v * e->n, 8 * (size_t)e->n, hipMemcpyDeviceToHost) == hipSuccess
             ? SWIM_OK : SWIM_EDEVICE;
}

int32_t swim_drain_events(swim_engine* e, swim_event* out, size_t cap, size_t* n_out) {
  if (!e || (cap && !out)) return SWIM_EINVAL;
  int32_t rc = sync_and_collect(e);
  if (rc == SWIM_EDEVICE) return rc;
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
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  unsigned long long st[ST_COUNT];
  if (read_stats(e, st) != SWIM_OK) return SWIM_EDEVICE;
  std::memset(out, 0, sizeof(*out));
  out->ticks = e->host_ticks;
  out->pings = st[ST_PINGS];
  out->ping_reqs = st[ST_PING_REQS];
  out->fd_events = st[ST_FD_EVENTS];
  out->gossips_created = st[ST_GOSSIPS_CREATED];
  out->gossip_messages = st[ST_GOSSIP_MESSAGES];
  out->gossip_accepted = st[ST_GOSSIP_ACCEPTED];
  out->syncs = st[ST_SYNCS];
  out->sync_acks = st[ST_SYNC_ACKS];
  out->sync_records = st[ST_SYNC_RECORDS];
  out->fetches = st[ST_FETCHES];
  out->fetch_ok = st[ST_FETCH_OK];
  out->timers_fired = st[ST_TIMERS_FIRED];
  out->events = e->host_events;
  out->capacity_errors = e->err_seen;
  return SWIM_OK;
}

int32_t swim_read_member(swim_engine* e, uint32_t v, swim_member_state* o) {
  if (!e || v >= e->n || !o) return SWIM_EINVAL;
  MemberDev m;
  if (read_member_dev(e, v, &m) != SWIM_OK) return SWIM_EDEVICE;
  std::memset(o, 0, sizeof(*o));
  o->up = m.up;
  o->joined = m.joined;
  o->leave_pending = m.leave_pending;
  o->join_pending = m.join_pending;
  o->remote_idx = m.remote_idx;
  o->fd_period = m.fd_period;
  o->ping_cursor = m.ping_cursor;
  o->ping_len = m.ping_len;
  o->remote_len = m.remote_len;
  o->gossip_len = m.gossip_len;
  o->gossip_period = m.g_period;
  o->gossip_counter = m.g_counter;
  o->table_size = m.table_size;
  o->members_size = m.members_size;
  o->fd_start = m.fd_start;
  o->gossip_start = m.g_start;
  o->sync_start = m.sync_start;
  o->sync_on = m.sync_on;
  o->ack_target = m.ack_due ? m.ack_target : 0xffffffffu;
  o->ack_due = m.ack_due;
  o->relay_target = m.relay_due ? m.relay_target : 0xffffffffu;
  o->relay_pending = m.relay_due ? m.relay_pending : 0;
  o->relay_due = m.relay_due;
  o->leave_gossiper = m.leave_pending ? m.leave_gossiper : 0xffffffffu;
  o->leave_seq = m.leave_pending ? m.leave_seq : 0;
  return SWIM_OK;
}

static int32_t read_list(swim_engine* e, uint32_t v, const uint32_t* base, uint32_t len, uint32_t* out, uint32_t cap,
                         uint32_t* lenp) {
  if (lenp) *lenp = len;
  if (out && cap && len) {
    uint32_t k = std::min(cap, len);
    if (hipMemcpy(out, base + (size_t)v * e->n, 4 * (size_t)k, hipMemcpyDeviceToHost) != hipSuccess) return SWIM_EDEVICE;
  }
  return SWIM_OK;
}

int32_t swim_read_ping_list(swim_engine* e, uint32_t v, uint32_t* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  MemberDev m;
  if (read_member_dev(e, v, &m) != SWIM_OK) return SWIM_EDEVICE;
  return read_list(e, v, e->c.ping, m.ping_len, out, cap, len);
}

int32_t swim_read_remote_list(swim_engine* e, uint32_t v, uint32_t* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  MemberDev m;
  if (read_member_dev(e, v, &m) != SWIM_OK) return SWIM_EDEVICE;
  return read_list(e, v, e->c.remote, m.remote_len, out, cap, len);
}

int32_t swim_read_gossips(swim_engine* e, uint32_t v, swim_gossip* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  MemberDev m;
  if (read_member_dev(e, v, &m) != SWIM_OK) return SWIM_EDEVICE;
  if (len) *len = m.gossip_len;
  uint32_t k = std::min(cap, m.gossip_len);
  if (!out || !k) return SWIM_OK;
  std::vector<GossipDev> g(k);
  if (hipMemcpy(g.data(), e->c.slab + (size_t)v * e->c.gcap, sizeof(GossipDev) * k, hipMemcpyDeviceToHost) != hipSuccess)
    return SWIM_EDEVICE;
  for (uint32_t i = 0; i < k; ++i) {
    out[i].gossiper = g[i].gossiper;
    out[i].subject = g[i].subject;
    out[i].seq = g[i].seq;
    out[i].inc = g[i].inc;
    out[i].status = g[i].status;
    out[i].infection_period = g[i].inf_period;
    out[i].infected[0] = g[i].inf0;
    out[i].infected[1] = g[i].inf1;
  }
  return SWIM_OK;
}

int32_t swim_read_collector(swim_engine* e, uint32_t v, uint32_t gossiper, swim_interval* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  std::vector<CollDev> tab(e->c.hcap);
  if (hipMemcpy(tab.data(), e->c.coll + (size_t)v * e->c.hcap, sizeof(CollDev) * e->c.hcap, hipMemcpyDeviceToHost) !=
      hipSuccess)
    return SWIM_EDEVICE;
  if (len) *len = 0;
  for (const CollDev& d : tab) {
    if (d.key != gossiper + 1) continue;
    if (len) *len = d.n;
    for (uint32_t i = 0; i < d.n && i < cap && out; ++i) {
      out[i].lo = d.lo[i];
      out[i].hi = d.hi[i];
    }
    break;
  }
  return SWIM_OK;
}

int32_t swim_profile_enable(swim_engine* e, int32_t enable) {
  if (!e) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  if (e->prof_ev.empty()) {
    e->prof_ev.resize(4 * kDrainEvery + 4);
    for (auto& ev : e->prof_ev)
      if (hipEventCreate(&ev) != hipSuccess) return SWIM_EDEVICE;
  }
  e->prof_used = 0;
  e->prof_ms = 0;
  e->prof_launches = 0;
  unsigned long long st[ST_COUNT];
  if (read_stats(e, st) != SWIM_OK) return SWIM_EDEVICE;
  e->prof_base_msgs = st[ST_MERGE_MSGS];
  e->prof_base_recs = st[ST_MERGE_RECORDS];
  e->prof = enable != 0;
  return SWIM_OK;
}

int32_t swim_profile_merge(swim_engine* e, swim_kernel_profile* out) {
  if (!e || !out) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  prof_flush(e);
  unsigned long long st[ST_COUNT];
  if (read_stats(e, st) != SWIM_OK) return SWIM_EDEVICE;
  out->launches = e->prof_launches;
  out->total_ms = e->prof_ms;
  out->messages = st[ST_MERGE_MSGS] - e->prof_base_msgs;
  out->records = st[ST_MERGE_RECORDS] - e->prof_base_recs;
  out->alg_bytes = out->messages * (uint64_t)e->n * 16ull + out->records * 8ull;
  return SWIM_OK;
}

// ---- KAT hooks: run the device code paths on given inputs
int32_t swim_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  if (!ctr || !key || !out) return SWIM_EINVAL;
  uint32_t* d = nullptr;
  if (hipMalloc((void**)&d, 40) != hipSuccess) return SWIM_EDEVICE;
  hipMemcpy(d, ctr, 16, hipMemcpyHostToDevice);
  hipMemcpy(d + 4, key, 8, hipMemcpyHostToDevice);
  k_kat_philox<<<1, 64>>>(d, d + 4, d + 6);
  hipError_t r = hipMemcpy(out, d + 6, 16, hipMemcpyDeviceToHost);
  hipFree(d);
  return r == hipSuccess ? hip_status() : SWIM_EDEVICE;
}

int32_t swim_kat_overrides(const int32_t* cases, uint32_t n, uint8_t* out) {
  if (n && (!cases || !out)) return SWIM_EINVAL;
  if (!n) return SWIM_OK;
  int32_t* dc = nullptr;
  uint8_t* dout = nullptr;
  if (hipMalloc((void**)&dc, 20 * (size_t)n) != hipSuccess) return SWIM_EDEVICE;
  if (hipMalloc((void**)&dout, n) != hipSuccess) { hipFree(dc); return SWIM_EDEVICE; }
  hipMemcpy(dc, cases, 20 * (size_t)n, hipMemcpyHostToDevice);
  k_kat_overrides<<<grid_for(n, 256), 256>>>(dc, n, dout);
  hipError_t r = hipMemcpy(out, dout, n, hipMemcpyDeviceToHost);
  hipFree(dc);
  hipFree(dout);
  return r == hipSuccess ? hip_status() : SWIM_EDEVICE;
}

int32_t swim_kat_collector(const uint8_t* kinds, const int64_t* values, uint32_t n, int64_t* results) {
  if (n && (!kinds || !values || !results)) return SWIM_EINVAL;
  if (!n) return SWIM_OK;
  uint8_t* dk = nullptr;
  int64_t* dv = nullptr;
  int64_t* dr = nullptr;
  CollDev* de = nullptr;
  uint32_t* derr = nullptr;
  if (hipMalloc((void**)&dk, n) != hipSuccess || hipMalloc((void**)&dv, 8 * (size_t)n) != hipSuccess ||
      hipMalloc((void**)&dr, 8 * (size_t)n) != hipSuccess || hipMalloc((void**)&de, sizeof(CollDev)) != hipSuccess ||
      hipMalloc((void**)&derr, 4) != hipSuccess)
    return SWIM_EDEVICE;
  hipMemcpy(dk, kinds, n, hipMemcpyHostToDevice);
  hipMemcpy(dv, values, 8 * (size_t)n, hipMemcpyHostToDevice);
  hipMemset(derr, 0, 4);
  Ctx c{};
  c.err = derr;
  k_kat_collector<<<1, 64>>>(c, dk, dv, n, dr, de);
  hipError_t r = hipMemcpy(results, dr, 8 * (size_t)n, hipMemcpyDeviceToHost);
  uint32_t err = 0;
  hipMemcpy(&err, derr, 4, hipMemcpyDeviceToHost);
  hipFree(dk); hipFree(dv); hipFree(dr); hipFree(de); hipFree(derr);
  if (r != hipSuccess) return SWIM_EDEVICE;
  return err ? SWIM_ECAPACITY : hip_status();
}

}  // extern "C"
