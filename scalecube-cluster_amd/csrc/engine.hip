// engine.hip — host orchestration and C ABI (include/swim.h) of libswimgpu.so.
//
// A swim_engine simulates one cluster of N members whose view rows are sharded by viewer
// (DESIGN.md §7).  It holds the shards it runs in this process:
//   * unsharded (world = 1): one shard owning every row — the single-GPU engine;
//   * local group (cfg.local_shards = G > 1): all G shards in this process on one device (the
//     bit-exact test rig of the sharded path);
//   * RCCL (swim_create_shard): one shard per process / GPU, the other ranks' exchange regions
//     mapped over xGMI.
// Both multi-shard modes run the same device-side exchange: producers write into their own region,
// each shard learns on the device what every peer produced for it (ncclAllToAll of the counts, or
// k_gather_counts in a local group), and fixed-grid kernels pull the items (k_recv_msgs,
// k_recv_sync, k_pull_rows).
//
// Per tick every shard runs the kernel sequence of swim_phases.h on the engine's stream; no engine
// synchronises with the host inside a tick.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <new>
#include <vector>

#include "swim_phases.h"

using namespace swimdev;

namespace {

constexpr uint32_t kDrainEvery = 256;  // longest interval between event drains (ticks)
constexpr uint32_t kDrainFirst = 1;    // the interval starts at one tick and adapts to the event rate
#ifndef CLS_GRID
#define CLS_GRID 4096
#endif
constexpr uint32_t kClassifyGrid = CLS_GRID;  // 16,384 waves: about one (message, chunk) unit each at N = 65,536
constexpr uint32_t kApplyGrid = 256;      // grid-stride over receivers
#ifndef EMIT_GRID
#define EMIT_GRID 1024
#endif
// 4,096 waves, one gossip sender at a time each: all resident at the kernel's occupancy (4 waves per
// SIMD); 2,048 workgroups (two rounds of waves) measured 7 % slower in a storm, 512 8 % slower
constexpr uint32_t kEmitGrid = EMIT_GRID;
#ifndef DLV_GRID
#define DLV_GRID 512
#endif
constexpr uint32_t kDeliverGrid = DLV_GRID;  // 2,048 waves (two workgroups per CU) for the big inboxes of a storm
constexpr uint32_t kStopCap = 4096;
constexpr uint32_t kProfEvery = 3;  // SYNC classify launches between timed ones
constexpr uint64_t kRebaseEvery = 16;  // ticks between rebases of the SYNC block witness (k_end_tick)

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

uint32_t grid_for(uint32_t n, uint32_t block) { return std::max(1u, (n + block - 1) / block); }

}  // namespace

// One shard: the device state of rows [lo, lo + nl) plus the replicated arrays.
// One kernel's sampled launch timing: HIP events bound to the dispatch itself (hipExtLaunchKernelGGL:
// the kernel's own start / completion timestamps, no extra stream packets) on one launch in
// kProfEvery, plus three per-launch work counters the kernel accumulates into `slots`.
struct KProf {
  std::vector<hipEvent_t> ev;
  uint32_t used = 0;
  uint64_t seen = 0;  // launches since profiling was enabled
  unsigned long long* slots = nullptr;  // per sampled launch: {work counters a, b, c}
  double ms = 0;
  unsigned long long a = 0, b = 0, c = 0;
  uint64_t launches = 0;

  bool take(bool on) { return on && (seen++ % kProfEvery) == 0 && 2 * (used + 1) <= ev.size(); }
  void flush() {
    if (!used) return;
    std::vector<unsigned long long> h(3 * (size_t)used);
    hipMemcpy(h.data(), slots, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
    hipMemset(slots, 0, sizeof(unsigned long long) * h.size());
    for (uint32_t i = 0; i < used; ++i) {
      float t = 0.f;
      if (hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]) == hipSuccess) ms += t;
      a += h[3 * i];
      b += h[3 * i + 1];
      c += h[3 * i + 2];
    }
    launches += used;
    used = 0;
  }
  void reset() {
    hipMemset(slots, 0, sizeof(unsigned long long) * 3 * ev.size());
    used = 0;
    seen = 0;
    ms = 0;
    a = b = c = 0;
    launches = 0;
  }
};

struct Shard {
  Ctx c{};
  Bufs b{};
  Counters* k = nullptr;
  Xc* x = nullptr;
  std::vector<void*> allocs;
  // cross-shard exchange: the producer-side buffers (tx_msgs, tx_reqs, tx_acks,
  // tx_stops, tx_rows) live in one allocation, `xreg`, whose IPC handle the other ranks open;
  // `peers` (device) says where this shard reads what the others produced for it
  void* xreg = nullptr;
  size_t xreg_bytes = 0;
  bool xreg_uncached = false;  // the region came from hipDeviceMallocUncached
  void* rx_rows_h[2] = {nullptr, nullptr};  // the pulled-row copies Peers points at (RCCL / pull rig)
  uint32_t rx_row_cap = 0;                    // the row_cap they were sized for
  Peers* peers = nullptr;
  std::vector<void*> ipc_open;  // peers' regions mapped here (RCCL)
  uint32_t links_dev_cap = 0;
  size_t mseed_cap = 0;  // capacity of c.mseed (swim_set_member_seeds)
  uint64_t* delay_buf = nullptr;  // the delay threshold tables (Ctx.delay_th)
  size_t delay_cap = 0;           // words allocated
  // device-resident launch parameters (swim_phases.h Params) and the last uploaded image
  Params* d_par = nullptr;
  Params up{};
  bool up_valid = false;
  // swim_profile_*: HIP events around sampled k_sync_classify (merge) and k_gossip_emit (fanout)
  // launches on the engine's stream
  KProf prof_cls, prof_emit, prof_dlv;

  template <typename T>
  bool alloc(T** p, size_t count) {
    if (dalloc(p, count) != hipSuccess) return false;
    allocs.push_back((void*)*p);
    return true;
  }
  void release(void* p) {
    if (!p) return;
    allocs.erase(std::remove(allocs.begin(), allocs.end(), p), allocs.end());
    hipFree(p);
  }
  // (keep: the first *cap elements are copied into the new allocation; the caller has drained the stream)
  template <typename T>
  bool grow(T** p, size_t* cap, size_t need, bool keep = false) {
    if (need <= *cap) return true;
    size_t nc = std::max<size_t>(need, *cap * 2);
    T* q = nullptr;
    if (dalloc(&q, nc) != hipSuccess) return false;
    if (keep && *p && *cap && hipMemcpy(q, *p, sizeof(T) * *cap, hipMemcpyDeviceToDevice) != hipSuccess) return false;
    if (*p) {
      allocs.erase(std::remove(allocs.begin(), allocs.end(), (void*)*p), allocs.end());
      hipFree(*p);
    }
    *p = q;
    *cap = nc;
    allocs.push_back((void*)q);
    return true;
  }
};

struct swim_engine {
  swim_config cfg{};
  int debug_sync = 0;  // SWIM_DEBUG_SYNC=1: synchronise after every tick kernel and name a faulting one
  bool pull_rows = false;  // content rows pulled into local copies (RCCL; SWIM_EXCHANGE_PULL=1 in a local group)
  std::chrono::steady_clock::time_point debug_t{};
  int32_t device = 0;
  uint32_t n = 0, tick_ms = 0, P = 0, G = 0, S = 0, sz = 0;
  uint64_t T = 0;
  int32_t rank = 0, world = 1;  // this process's shard (RCCL) and the cluster's shard count
  bool rccl = false;
  bool rfilter_on = false;  // emit's cross-shard receipt filter (local groups, setup_peers_local)
  uint32_t xflags = 0;  // SWIM_XCHG_IPC* (swim_exchange_info): which branch of setup_peers_rccl ran
  bool xchg = false;  // the exchange machinery runs: world > 1, or RCCL with one rank (swim_create_shard)
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  std::vector<Shard> sh;  // local shards, in shard order
  uint32_t* d_cnt = nullptr;  // RCCL: the capacity-error allreduce of swim_step_ticks
  Params* h_par = nullptr;    // pinned staging ring for Params uploads
  uint32_t par_slot = 0;
  // host mirrors of replicated control state
  std::vector<uint8_t> g_residue;  // gossip timer residues mod G in use
  uint32_t drain_every = kDrainFirst, since_drain = 0;  // event drain interval (ticks), adaptive
  std::vector<uint32_t> seeds;
  // per-member seedMembers (swim_set_member_seeds): own list of each member (mseed_own_h), uploaded
  // as CSR to every shard before the next step when changed
  std::vector<std::vector<uint32_t>> mseeds_h;
  std::vector<uint8_t> mseed_own_h;
  bool mseed_dirty = false;
  std::vector<uint8_t> is_seed_h, joined_h, join_pending_h;
  std::vector<LinkDev> links_h;
  std::vector<int32_t> delay_means;  // NetworkEmulator meanDelay (ms) of each delay table, in table order
  std::vector<uint32_t> joins;  // joins starting at the next tick
  std::vector<std::pair<uint64_t, uint32_t>> fq_joins;  // (tick, joiner) of the recent joins (grow_for_joins)
  // addresses (swim_join_at): addr_h[x] = the address member x was started on, route_h[x] = the
  // member listening on it now (both empty while every member is on its own address); binds: the
  // (joiner, member whose address it takes) pairs starting at the next tick
  std::vector<uint32_t> addr_h, route_h;
  std::vector<std::pair<uint32_t, uint32_t>> binds;
  uint32_t route_of(uint32_t x) const { return route_h.empty() ? x : route_h[x]; }
  std::vector<swim_event> events;
  uint64_t host_ticks = 0, host_events = 0;
  uint32_t row_grows = 0;  // times row_cap grew before a join burst (grow_rows_for_joins)
  // quiet windows (swim_quiet.h): on unless disabled; after a window that advanced nothing, the next
  // try waits quiet_backoff ticks (doubling), so a busy cluster pays a scan only now and then
  bool quiet_on = true;
  QuietCtl* d_quiet = nullptr;   // [2] device control blocks (shared by the local shards), alternating
  uint32_t q_par = 0;            // the block the next window uses
  // the next window precomputed by a window's apply (swim_quiet.h QuietPre): [2] tagged keys
  // (alternating), the tag of the last one written, and whether it still holds: for the window that
  // starts at pre_T0 with at most pre_H ticks, and nothing but quiet windows ran since (pre_valid is
  // cleared by every per-tick tick and every API call that changes state or configuration: mutated())
  uint64_t* d_pre = nullptr;
  uint32_t pre_tag = 0, pre_slot = 0, pre_H = 0;
  uint64_t pre_T0 = 0;
  bool pre_valid = false;
  bool pre_on = true;            // SWIM_QUIET_PRE=0: every window scans
  uint32_t* h_stat = nullptr;    // pinned host words: each local shard's event counts and error bits
  uint32_t* d_stat = nullptr;    //   ([SUBQ + 1] per shard, written by k_status), and their device address
  uint32_t* h_done = nullptr;    // pinned host words: the last window's length (written by k_quiet_apply),
                                 //   [1] k_status's sequence number (the window's wait, wait_status_seq)
  uint32_t status_seq = 0;
  // no member has ever stopped (kill, graceful leave) or been given an inbound filter, and no
  // external record was ingested: every member a ping list can hold is up and lets pings in, so a
  // quiet window's pings need no target check (k_quiet_scan `pingable`)
  bool pristine = true;
  bool spin_wait = true;         // SWIM_SPIN=0: the window waits with hipStreamSynchronize
  uint32_t* d_done = nullptr;    // its device address
  uint32_t* d_refmm = nullptr;   // RCCL: [2][n] elementwise min / max of the ranks' witness refs
  uint64_t quiet_retry_at = 0;
  uint32_t quiet_backoff = 1;
  swim_quiet_stats qst{};
  // swim_profile_quiet: HIP events around every window's kernels (scan .. apply) while profiling
  // (a ring of event pairs, read when the profile is read or the ring is full: a window's own wait
  // never synchronises on an event, which would put the runtime's completion signalling into the
  // measured call)
  static constexpr uint32_t kQevRing = 64;
  hipEvent_t qev[2 * kQevRing] = {};
  uint32_t qev_n = 0;            // pairs recorded and not yet read
  double qprof_ms = 0.0;
  uint64_t qprof_windows = 0, qprof_ticks = 0, qprof_mp = 0, qprof_bytes = 0;
  std::vector<uint8_t> loss_h;   // host mirror of the default outbound loss per member
  uint32_t loss_nz = 0;          // members whose default loss is not 0
  uint32_t err_seen = 0;
  bool prof = false;

  ~swim_engine() {
    if (stream) hipStreamSynchronize(stream);
    for (Shard& s : sh) {
      for (hipEvent_t ev : s.prof_cls.ev) hipEventDestroy(ev);
      for (hipEvent_t ev : s.prof_emit.ev) hipEventDestroy(ev);
      for (hipEvent_t ev : s.prof_dlv.ev) hipEventDestroy(ev);
      for (void* p : s.ipc_open) hipIpcCloseMemHandle(p);
      for (void* p : s.allocs) hipFree(p);
      if (s.xreg) hipFree(s.xreg);
    }
    if (d_cnt) hipFree(d_cnt);
    if (d_quiet) hipFree(d_quiet);
    if (d_pre) hipFree(d_pre);
    if (d_refmm) hipFree(d_refmm);
    for (hipEvent_t ev : qev)
      if (ev) hipEventDestroy(ev);
    if (h_done) hipHostFree(h_done);
    if (h_stat) hipHostFree(h_stat);
    if (h_par) hipHostFree(h_par);
    if (comm) ncclCommDestroy(comm);
    if (stream) hipStreamDestroy(stream);
  }
  // the local shard owning member v, or nullptr (RCCL: owned by another process)
  Shard* owner_of(uint32_t v) {
    const uint32_t o = v / sz;
    if (!rccl) return &sh[o];
    return (int32_t)o == rank ? &sh[0] : nullptr;
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

static int32_t nccl_ok(ncclResult_t r) {
  if (r == ncclSuccess) return SWIM_OK;
  std::fprintf(stderr, "libswimgpu: RCCL error %s\n", ncclGetErrorString(r));
  return SWIM_EDEVICE;
}

// device counters are replicated ST_REPL times; sum them over every local shard
static int32_t read_stats(swim_engine* e, unsigned long long* st) {
  std::vector<unsigned long long> rep((size_t)ST_COUNT * ST_REPL);
  for (int s = 0; s < ST_COUNT; ++s) st[s] = 0;
  for (Shard& sd : e->sh) {
    if (hipMemcpy(rep.data(), sd.c.stats, sizeof(unsigned long long) * rep.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return SWIM_EDEVICE;
    for (int s = 0; s < ST_COUNT; ++s)
      for (int r = 0; r < ST_REPL; ++r) st[s] += rep[(size_t)s * ST_REPL + r];
  }
  return SWIM_OK;
}

// The SYNC classify launch (the HBM stream) and the gossip fanout launch are sampled by KProf.
// The SYNC_ACK classify launch is a separate kernel (k_ack_classify).
static void launch_classify(swim_engine* e, Shard& s, int d2) {
  if (d2) {
    k_ack_classify<<<kClassifyGrid, CLS_BLOCK, 0, e->stream>>>(s.d_par, e->T);
    return;
  }
  KProf& k = s.prof_cls;
  if (!k.take(e->prof)) {
    k_sync_classify<<<kClassifyGrid, CLS_BLOCK, 0, e->stream>>>(s.d_par, e->T, nullptr);
    return;
  }
  hipExtLaunchKernelGGL(k_sync_classify, dim3(kClassifyGrid), dim3(CLS_BLOCK), 0, e->stream, k.ev[2 * k.used],
                        k.ev[2 * k.used + 1], 0, s.d_par, e->T, k.slots + 3 * k.used);
  k.used++;
}

static void launch_emit(swim_engine* e, Shard& s) {
  KProf& k = s.prof_emit;
  if (!k.take(e->prof)) {
    k_gossip_emit<<<kEmitGrid, 64 * EMIT_WAVES, 0, e->stream>>>(s.d_par, e->T, nullptr);
    return;
  }
  hipExtLaunchKernelGGL(k_gossip_emit, dim3(kEmitGrid), dim3(64 * EMIT_WAVES), 0, e->stream, k.ev[2 * k.used],
                        k.ev[2 * k.used + 1], 0, s.d_par, e->T, k.slots + 3 * k.used);
  k.used++;
}

// the fused SYNC apply (unsharded) carries the merge profile that k_sync_classify carries otherwise
static void launch_apply(swim_engine* e, Shard& s, int d2, int classified, int fused) {
  KProf& k = s.prof_cls;
  if (d2) {
    k_ack_apply<<<kApplyGrid, APPLY_BLOCK, 0, e->stream>>>(s.d_par, e->T, classified);
    return;
  }
  if (!fused || !k.take(e->prof)) {
    k_sync_apply<<<kApplyGrid, APPLY_BLOCK, 0, e->stream>>>(s.d_par, e->T, classified, fused, nullptr);
    return;
  }
  hipExtLaunchKernelGGL(k_sync_apply, dim3(kApplyGrid), dim3(APPLY_BLOCK), 0, e->stream, k.ev[2 * k.used],
                        k.ev[2 * k.used + 1], 0, s.d_par, e->T, classified, fused, k.slots + 3 * k.used);
  k.used++;
}

static void launch_deliver(swim_engine* e, Shard& s) {
  // at least kDeliverGrid workgroups: big inboxes are delivered a wave each, grid-stride
  // (the whole-wave delivery of the biggest inboxes first, its own kernel; both are "deliver" in the
  // profile: the events bracket the pair)
  const uint32_t grid = std::max<uint32_t>(kDeliverGrid, grid_for(s.c.nl, DLV_BLOCK));
  KProf& k = s.prof_dlv;
  if (!k.take(e->prof)) {
    k_deliver_coop<<<kDeliverGrid, DLV_BLOCK, 0, e->stream>>>(s.d_par, e->T, nullptr);
    k_gossip_deliver<<<grid, DLV_BLOCK, 0, e->stream>>>(s.d_par, e->T, 1, nullptr);
    return;
  }
  hipExtLaunchKernelGGL(k_deliver_coop, dim3(kDeliverGrid), dim3(DLV_BLOCK), 0, e->stream, k.ev[2 * k.used], nullptr,
                        0, s.d_par, e->T, k.slots + 3 * k.used);
  hipExtLaunchKernelGGL(k_gossip_deliver, dim3(grid), dim3(DLV_BLOCK), 0, e->stream, nullptr,
                        k.ev[2 * k.used + 1], 0, s.d_par, e->T, 1, k.slots + 3 * k.used);
  k.used++;
}

// each shard's event counts and error bits into the pinned host words (one launch instead of two
// blocking copies per shard: the drain that ends every swim_step call, quiet windows included)
// (seq_out, seq: the last shard's launch also publishes a sequence number after its words: a host
// that sees it knows every earlier kernel of the stream has completed — the quiet window's wait)
__global__ void k_status(const uint32_t* ev_cnt, const uint32_t* err, uint32_t* out, uint32_t* seq_out, uint32_t seq) {
  const uint32_t t = threadIdx.x;
  if (t < SUBQ) out[t] = ev_cnt[t];
  if (t == SUBQ) out[SUBQ] = *err;
  if (seq_out) {
    __syncthreads();
    if (t == 0) {
      __threadfence_system();
      __hip_atomic_store(seq_out, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

static void launch_status(swim_engine* e, uint32_t seq = 0) {
  for (size_t i = 0; i < e->sh.size(); ++i)
    k_status<<<1, 64, 0, e->stream>>>(e->sh[i].c.ev_cnt, e->sh[i].c.err, e->d_stat + i * (SUBQ + 1),
                                      seq && i + 1 == e->sh.size() ? e->d_done + 1 : nullptr, seq);
}
// the quiet window's wait: spin on the pinned sequence word k_status publishes (no runtime
// synchronisation: the sleep / wake-up of hipStreamSynchronize is most of a short window's host
// time); a stream error ends the spin (hipStreamQuery every 1,024 polls)
static int32_t wait_status_seq(swim_engine* e, uint32_t seq) {
  for (uint32_t it = 1;; ++it) {
    if (__atomic_load_n(e->h_done + 1, __ATOMIC_ACQUIRE) == seq) return SWIM_OK;
    if ((it & 1023u) == 0) {
      const hipError_t q = hipStreamQuery(e->stream);
      if (q == hipSuccess) return __atomic_load_n(e->h_done + 1, __ATOMIC_ACQUIRE) == seq ? SWIM_OK : SWIM_EDEVICE;
      if (q != hipErrorNotReady) return SWIM_EDEVICE;
    }
    __builtin_ia32_pause();
  }
}
// fresh: the status words were written by the last work on the stream and the stream has drained
// (a quiet window launches k_status before its own synchronisation): no launch, no second wait
static int32_t sync_and_collect(swim_engine* e, bool fresh = false) {
  if (!fresh) {
    launch_status(e);
    if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  }
  e->par_slot = 0;  // every staged Params upload has completed
  uint32_t err_all = 0;
  double fill = 0.0;  // fullest event sub-queue since the last drain
  for (size_t si = 0; si < e->sh.size(); ++si) {
    Shard& s = e->sh[si];
    uint32_t cnt[SUBQ], err = 0;
    const volatile uint32_t* st = e->h_stat + si * (SUBQ + 1);
    for (uint32_t q = 0; q < SUBQ; ++q) cnt[q] = st[q];
    err = st[SUBQ];
    bool any = false;
    for (uint32_t q = 0; q < SUBQ; ++q) {
      const uint32_t k = std::min(cnt[q], s.c.ev_cap);
      fill = std::max(fill, (double)cnt[q] / s.c.ev_cap);
      if (!k) continue;
      any = true;
      size_t old = e->events.size();
      e->events.resize(old + k);
      if (hipMemcpy(e->events.data() + old, s.c.ev + (size_t)q * s.c.ev_cap, sizeof(swim_event) * k,
                    hipMemcpyDeviceToHost) != hipSuccess)
        return SWIM_EDEVICE;
      e->host_events += k;
    }
    if (any && hipMemset(s.c.ev_cnt, 0, 4 * SUBQ) != hipSuccess) return SWIM_EDEVICE;
    err_all |= err;
    if (e->prof) {
      s.prof_cls.flush();
      s.prof_emit.flush();
      s.prof_dlv.flush();
    }
  }
  // adapt the drain interval so a sub-queue stays well below its capacity between drains (an event
  // storm — a join burst adds every joiner at every viewer — drains every few ticks, a quiet
  // cluster every kDrainEvery)
  if (fill > 0.5) e->drain_every = std::max(1u, e->drain_every / 4);
  else if (fill > 0.25) e->drain_every = std::max(1u, e->drain_every / 2);
  else if (fill < 0.05) e->drain_every = std::min(kDrainEvery, e->drain_every * 2);
  e->since_drain = 0;
  e->err_seen |= err_all;
  return err_all ? SWIM_ECAPACITY : SWIM_OK;
}

// ------------------------------------------------------------------------------- exchange
// Per exchange (E1 GOSSIP_REQs + stops, E2 SYNCs, E3 SYNC_ACKs) every shard learns, on the device,
// how many items each other shard produced for it, then pulls them from the producers' buffers with
// kernels that read those counts themselves: no host synchronisation and no copies
// sized by the host.  RCCL: one ncclAllToAll of the per-destination counts (+ one ncclAllGather of
// the stop counts on E1), which is also the barrier after which the producers' buffers are complete;
// a local group: k_gather_counts reads the peer shards' counters.
constexpr uint32_t kRecvGrid = 1024, kPackGrid = 2048;

static int32_t exchange_counts(swim_engine* e, uint32_t kind) {
  hipStream_t s = e->stream;
  if (e->rccl) {
    Shard& sd = e->sh[0];
    uint32_t* send = kind == XK_MSG ? sd.x->msg : kind == XK_REQ ? sd.x->req : sd.x->ack;
    if (ncclGroupStart() != ncclSuccess) return SWIM_EDEVICE;
    ncclAllToAll(send, sd.b.rx_cnt + kind * MAXW, 1, ncclUint32, e->comm, s);
    if (kind == XK_MSG) ncclAllGather(&sd.x->stop, sd.b.rx_cnt + XK_STOP * MAXW, 1, ncclUint32, e->comm, s);
    return nccl_ok(ncclGroupEnd());
  }
  for (Shard& sd : e->sh) k_gather_counts<<<1, 64, 0, s>>>(sd.d_par, e->T, (int)kind);
  return SWIM_OK;
}

static Ctx sync_ctx(Shard& sd) {  // list inserts of the SYNC phase use the second set of counters
  Ctx cd = sd.c;
  cd.ins_total = &sd.k->ins_total2;
  return cd;
}

// Upload the shard's launch parameters when any field differs from the image the device holds.
// Uploads go through a pinned staging ring on the engine's stream, so they are ordered with the
// kernels; the ring wraps only after a stream synchronisation.
constexpr uint32_t kParRing = 64;
static void sync_params(swim_engine* e, Shard& sd) {
  Params p;
  std::memset(&p, 0, sizeof p);
  p.c = sd.c;
  p.cs = sync_ctx(sd);
  p.b = sd.b;
  p.c.T = p.cs.T = 0;  // the tick travels as a kernel argument
  if (sd.up_valid && std::memcmp(&p, &sd.up, sizeof p) == 0) return;
  if (e->par_slot == kParRing) {
    hipStreamSynchronize(e->stream);
    e->par_slot = 0;
  }
  Params* stage = e->h_par + e->par_slot++;
  std::memcpy(stage, &p, sizeof p);
  hipMemcpyAsync(sd.d_par, stage, sizeof p, hipMemcpyHostToDevice, e->stream);
  sd.up = p;
  sd.up_valid = true;
}


// SWIM_DEBUG_SYNC=1: synchronise after each tick kernel so a device fault names its kernel;
// SWIM_DEBUG_SYNC=2 also names every kernel that took longer than 20 ms (wall, after the sync)
static void debug_slow(swim_engine* e, const char* name, uint64_t T);
#define TICK_CHECK(name)                                                                            \
  do {                                                                                              \
    if (e->debug_sync && hipStreamSynchronize(s) != hipSuccess) {                                   \
      std::fprintf(stderr, "libswimgpu: %s faulted at tick %llu\n", name, (unsigned long long)T);  \
      return SWIM_EDEVICE;                                                                          \
    }                                                                                               \
    if (e->debug_sync > 1) debug_slow(e, name, T);                                                  \
  } while (0)
static void debug_slow(swim_engine* e, const char* name, uint64_t T) {
  const auto now = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(now - e->debug_t).count();
  if (ms > 20.0) std::fprintf(stderr, "libswimgpu: %s took %.1f ms at tick %llu\n", name, ms, (unsigned long long)T);
  e->debug_t = now;
}

// One tick: 7 kernels per shard (11 on gossip ticks); a sharded engine adds k_recv_* and three exchanges.
// joiners of this tick that take another member's address start listening on it: route_h is
// recomputed and copied to every shard's replicated Ctx.route (allocated at the first bind)
static int32_t apply_binds(swim_engine* e) {
  if (e->route_h.empty()) {
    e->route_h.resize(e->n);
    e->addr_h.resize(e->n);
    for (uint32_t x = 0; x < e->n; ++x) e->route_h[x] = e->addr_h[x] = x;
  }
  for (auto& bd : e->binds) {
    const uint32_t A = e->addr_h[bd.second];
    e->addr_h[bd.first] = A;
    for (uint32_t x = 0; x < e->n; ++x)
      if (e->addr_h[x] == A) e->route_h[x] = bd.first;
  }
  e->binds.clear();
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  for (Shard& sd : e->sh) {
    if (!sd.c.route) {
      uint32_t* r = nullptr;
      if (!sd.alloc(&r, e->n)) return SWIM_ENOMEM;
      sd.c.route = r;
    }
    if (hipMemcpy((void*)sd.c.route, e->route_h.data(), 4 * (size_t)e->n, hipMemcpyHostToDevice) != hipSuccess)
      return SWIM_EDEVICE;
  }
  return SWIM_OK;
}

// row_cap — the content rows one shard may send in one SYNC (or SYNC_ACK) exchange — grows before a
// tick whose joins could exceed it: every joiner sends its initial SYNC to every seed
// (MembershipProtocolImpl.start0 :250-291) and each seed answers every one, so a join burst needs up
// to (joins on a shard) x seeds rows on the joiners' side and joins x (seeds on a shard) on the seeds'
// side, on top of the periodic SYNCs.  Only replicated control state decides (the pending joins, the
// seeds), so every RCCL rank grows at the same tick and all of them enter the re-exchange of the
// regions' IPC handles.  Rows are bounded at 4 GiB per direction.
static int32_t alloc_xreg(swim_engine* e, Shard& sd, bool uncached);
static int32_t setup_peers_local(swim_engine* e);
static int32_t setup_peers_rccl(swim_engine* e);
// the minimum of x over the RCCL ranks (x itself on a local group)
static int32_t rank_min(swim_engine* e, uint32_t& x) {
  if (!e->rccl) return SWIM_OK;
  if (hipMemcpy(e->d_cnt, &x, 4, hipMemcpyHostToDevice) != hipSuccess ||
      nccl_ok(ncclAllReduce(e->d_cnt, e->d_cnt + 1, 1, ncclUint32, ncclMin, e->comm, e->stream)) != SWIM_OK ||
      hipStreamSynchronize(e->stream) != hipSuccess || hipMemcpy(&x, e->d_cnt + 1, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return SWIM_EDEVICE;
  return SWIM_OK;
}
static size_t xreg_bytes_for(const swim_engine* e, const Bufs& b, uint32_t row_cap);
static void* xreg_alloc(size_t bytes, bool uncached, bool* got_uncached = nullptr);
static int32_t xreg_install(swim_engine* e, Shard& sd, void* fresh, uint32_t row_cap);
static int32_t grow_rows_for_joins(swim_engine* e) {
  if (!e->xchg || e->joins.empty() || e->sh.empty()) return SWIM_OK;
  const uint32_t W = (uint32_t)e->world;
  std::vector<uint64_t> jn(W, 0), sn(W, 0);
  for (uint32_t m : e->joins) jn[std::min(W - 1, m / e->sz)]++;
  for (uint32_t x : e->seeds) sn[std::min(W - 1, x / e->sz)]++;
  const uint64_t J = e->joins.size(), S = std::max<uint64_t>(1, e->seeds.size());
  uint64_t need = 0;
  for (uint32_t p = 0; p < W; ++p) need = std::max({need, jn[p] * S, J * sn[p]});
  need += 64 + (uint64_t)e->sz / std::max(e->S, 1u);  // the tick's periodic SYNCs beside them
  const uint32_t cur = e->sh[0].b.row_cap;
  uint64_t cap = cur;
  while (cap < need) cap *= 2;
  cap = std::min<uint64_t>(cap, std::max<uint64_t>(cur, (4ull << 30) / (4ull * e->n)));
  if (cap <= cur) return SWIM_OK;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  // what the grown rows cost, beside the regions in use (they are released only once every rank has
  // its new ones): both tx row regions and, where rows are pulled, the per-peer copies
  const bool pulled = e->rccl || e->pull_rows;
  const auto bytes_for = [&](uint64_t k) {
    uint64_t b = 0;
    for (const Shard& sd : e->sh) b += xreg_bytes_for(e, sd.b, (uint32_t)k) + (pulled ? 2ull * W * k * e->n * 4 : 0);
    return b;
  };
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return SWIM_EDEVICE;
  while (cap > cur && bytes_for(cap) > fr - fr / 8) cap /= 2;
  // every rank agrees on the size before anything changes (the inputs above differ by rank)
  uint32_t c32 = (uint32_t)cap;
  if (int32_t rc = rank_min(e, c32)) return rc;
  cap = c32;
  if (cap <= cur) return SWIM_OK;  // no room: the rows stay (a tick that overflows them reports ERR_REQS)
  // 1. the new regions and pulled copies, the old ones still in place
  std::vector<void*> fresh(e->sh.size(), nullptr);
  std::vector<std::array<uint32_t*, 2>> rx(e->sh.size(), {nullptr, nullptr});
  uint32_t ok = 1;
  for (size_t i = 0; i < e->sh.size() && ok; ++i) {
    fresh[i] = xreg_alloc(xreg_bytes_for(e, e->sh[i].b, (uint32_t)cap), e->rccl, &e->sh[i].xreg_uncached);
    ok = fresh[i] != nullptr;
    for (int k = 0; k < 2 && ok && pulled; ++k)
      ok = dalloc(&rx[i][k], (size_t)W * cap * e->n) == hipSuccess;
  }
  const auto release_fresh = [&](size_t from) {
    for (size_t i = from; i < e->sh.size(); ++i) {
      if (fresh[i]) hipFree(fresh[i]);
      for (uint32_t* q : rx[i])
        if (q) hipFree(q);
    }
  };
  if (int32_t rc = rank_min(e, ok)) {
    release_fresh(0);
    return rc;
  }
  if (!ok) {  // some rank could not: every rank keeps its region and row_cap
    release_fresh(0);
    return SWIM_OK;
  }
  // 2. every rank unmaps the others' regions before any region is freed
  if (e->rccl) {
    Shard& sd = e->sh[0];
    for (void* q : sd.ipc_open) hipIpcCloseMemHandle(q);
    sd.ipc_open.clear();
    if (nccl_ok(ncclAllReduce(e->d_cnt, e->d_cnt, 1, ncclUint32, ncclMax, e->comm, e->stream)) != SWIM_OK ||
        hipStreamSynchronize(e->stream) != hipSuccess) {
      release_fresh(0);
      return SWIM_EDEVICE;
    }
  }
  // 3. the switch: headers carried over, old regions and copies released
  for (size_t i = 0; i < e->sh.size(); ++i) {
    Shard& sd = e->sh[i];
    if (int32_t rc = xreg_install(e, sd, fresh[i], (uint32_t)cap)) {
      release_fresh(i);  // (shards before i switched; the device is unusable anyway)
      return rc;
    }
    if (pulled)
      for (int k = 0; k < 2; ++k) {
        sd.release(sd.rx_rows_h[k]);
        sd.allocs.push_back(rx[i][k]);
        sd.rx_rows_h[k] = rx[i][k];
      }
    sd.rx_row_cap = (uint32_t)cap;
  }
  e->row_grows++;
  return e->rccl ? setup_peers_rccl(e) : setup_peers_local(e);
}

// Join bursts size two per-shard structures whose need the reference does not bound (grow_for_joins,
// before a tick that starts joins; the joins of the last 4 metadataTimeout spans are counted):
// * the delayed metadata queue (Ctx.fq, per tick parity) holds every GET_METADATA round trip in
//   flight on the shard.  Its base capacity, max(4096, 2n), covers the admissions of a cluster that
//   is not joining; a join adds up to n round trips on its own shard (its first SYNC_ACK admits the
//   whole table) and one per viewer of every shard (the joiner's admission, as the news spreads),
//   each in flight for at most metadataTimeout after its send;
// * the pending SYNC_ACKs of a member (Ctx.pa, pa_cap per member): a seed answers every joiner's
//   SYNC after the admission fetches it waits on, so a burst of J joiners through one seed holds J
//   of them at once beside the base PA_CAP.
// The live entries keep their slots.  Shard-local (no collective): an allocation that fails keeps the
// structure, and a tick that overflows it reports ERR_FETCHQ / ERR_PACK, never a silent drop.
static int32_t grow_for_joins(swim_engine* e) {
  if (e->joins.empty() || e->sh.empty()) return SWIM_OK;
  const uint64_t span = 4ull * ((e->sh[0].c.metadata_timeout + e->tick_ms - 1) / e->tick_ms) + 1;
  e->fq_joins.erase(std::remove_if(e->fq_joins.begin(), e->fq_joins.end(),
                                   [&](const std::pair<uint64_t, uint32_t>& j) { return j.first + span < e->T; }),
                    e->fq_joins.end());
  for (uint32_t m : e->joins) e->fq_joins.push_back({e->T, m});
  bool synced = false;
  const uint64_t pa_need = PA_CAP + e->fq_joins.size();
  for (Shard& sd : e->sh) {
    if (pa_need > sd.c.pa_cap) {
      const uint64_t cur = sd.c.pa_cap, rows = std::max(sd.c.nl, 1u);
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) != hipSuccess) return SWIM_EDEVICE;
      const uint64_t cap = std::min<uint64_t>(std::max(pa_need, 2 * cur), fr / 8 / (rows * sizeof(PAck)));
      PAck* q = nullptr;
      if (cap > cur) {
        if (!synced) {
          if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
          synced = true;
        }
        if (dalloc(&q, rows * cap) != hipSuccess) {
          (void)hipGetLastError();
        } else {
          if (hipMemcpy2D(q, cap * sizeof(PAck), sd.c.pa, cur * sizeof(PAck), cur * sizeof(PAck), rows,
                          hipMemcpyDeviceToDevice) != hipSuccess)
            return SWIM_EDEVICE;
          sd.release(sd.c.pa);
          sd.allocs.push_back(q);
          sd.c.pa = q;
          sd.c.pa_cap = (uint32_t)cap;
        }
      }
    }
    if (!sd.c.delay_on) continue;
    uint64_t need = std::max<uint64_t>(4096, 2ull * e->n);
    for (const auto& j : e->fq_joins) need += sd.c.nl + (e->owner_of(j.second) == &sd ? e->n : 0u);
    const uint64_t cur = sd.c.fq_cap;
    if (need <= cur) continue;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return SWIM_EDEVICE;
    const uint64_t cap = std::min<uint64_t>({std::max<uint64_t>(need, 2 * cur), fr / 8 / (2 * sizeof(FetchEnt)), NONE - 1});
    if (cap <= cur) continue;
    if (!synced) {
      if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
      synced = true;
    }
    FetchEnt* q = nullptr;
    if (dalloc(&q, 2 * cap) != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    for (int p = 0; p < 2; ++p)
      if (hipMemcpy(q + p * cap, sd.c.fq + p * cur, sizeof(FetchEnt) * cur, hipMemcpyDeviceToDevice) != hipSuccess)
        return SWIM_EDEVICE;
    sd.release(sd.c.fq);
    sd.allocs.push_back(q);
    sd.c.fq = q;
    sd.c.fq_cap = (uint32_t)cap;
  }
  return SWIM_OK;
}

static int32_t run_tick(swim_engine* e) {
  e->T += 1;
  e->host_ticks += 1;
  e->pre_valid = false;
  hipStream_t s = e->stream;
  if (!e->binds.empty())
    if (int32_t rc = apply_binds(e)) return rc;
  if (int32_t rc = grow_rows_for_joins(e)) return rc;
  if (int32_t rc = grow_for_joins(e)) return rc;
  const uint64_t T = e->T;
  const bool multi = e->xchg;
  const bool gossip_tick = e->g_residue[e->T % e->G] != 0;
  for (Shard& sd : e->sh) {
    sd.c.T = e->T;
    sync_params(e, sd);
  }
  if (e->debug_sync && multi) {  // the exchange pointers of a sharded tick are set
    for (Shard& sd : e->sh) k_debug_exchange<<<1, 64, 0, s>>>(sd.d_par, T);
    if (hipStreamSynchronize(s) != hipSuccess) return SWIM_EDEVICE;
    for (Shard& sd : e->sh) {
      uint32_t err = 0;
      if (hipMemcpy(&err, sd.c.err, 4, hipMemcpyDeviceToHost) != hipSuccess) return SWIM_EDEVICE;
      if (err & ERR_XPTR) {
        std::fprintf(stderr, "libswimgpu: shard %u: null exchange pointer at tick %llu\n", sd.c.rank,
                     (unsigned long long)T);
        return SWIM_EDEVICE;
      }
    }
  }
  if (!e->joins.empty()) {
    for (Shard& sd : e->sh)
      for (uint32_t m : e->joins) hipMemsetAsync(sd.c.up + m, 1, 1, s);
    for (Shard& sd : e->sh) {
      k_start_joins<<<grid_for(sd.c.nl, 256), 256, 0, s>>>(sd.d_par, T);
      TICK_CHECK("k_start_joins");
    }
    e->joins.clear();
  }
  // (every shard's FETCH / timers / FD / gossip-round setup before any shard's emit: the cross-shard
  // receipt filter reads the other shards' collector clears of this tick, as the unsharded emit sees
  // every member's)
  for (Shard& sd : e->sh) {
    const uint32_t gm = grid_for(sd.c.nl, 256);
    // ---- A: suspicion timeouts, B: list compaction of their REMOVED + failure detector
    // ---- C: gossip round (period++ and the sender list in k_fd, then emit)
    // with message delay every tick may deliver GOSSIP_REQs, so the SYNC collection that follows a
    // member's deliveries moves into k_gossip_deliver on every tick
    const bool delay = sd.c.delay_on != 0;
    if (delay) {  // ---- the FETCH phase: delayed metadata round trips arriving now
      k_fetch_due<<<gm, 256, 0, s>>>(sd.d_par, T);
      TICK_CHECK("k_fetch_due");
    }
    k_fd<<<gm, 256, 0, s>>>(sd.d_par, T, gossip_tick ? 1 : 0, gossip_tick || delay ? 0 : 1);
    TICK_CHECK("k_fd");
  }
  for (Shard& sd : e->sh) {
    if (gossip_tick) {
      launch_emit(e, sd);
      TICK_CHECK("k_gossip_emit");
    }
    if (sd.c.delay_on) {
      k_dq_release<<<(sd.b.dq_bcap + 255) / 256, 256, 0, s>>>(sd.d_par, T);
      TICK_CHECK("k_dq_release");
    }
  }
  if (gossip_tick || e->sh[0].c.delay_on) {
    if (multi)
      if (int32_t rc = exchange_counts(e, XK_MSG)) return rc;
    for (Shard& sd : e->sh) {
      if (multi) {
        k_recv_msgs<<<kRecvGrid, 256, 0, s>>>(sd.d_par, T);
        TICK_CHECK("k_recv_msgs");
      }
      launch_deliver(e, sd);
      TICK_CHECK("k_gossip_deliver");  // (also applies the phase's pingMembers inserts)
    }
  }
  // ---- D: SYNC / SYNC_ACK
  // (SYNC requests were collected by k_gossip_deliver on gossip ticks, by k_fd on the others)
  if (e->sh[0].c.delay_on)  // delayed SYNCs: contents parked, arrivals into the inboxes / the exchange
    for (Shard& sd : e->sh) {
      k_sync_delay<<<256, 256, 0, s>>>(sd.d_par, T);
      TICK_CHECK("k_sync_delay");
    }
  for (int d2 = 0; d2 < 2; ++d2) {
    if (multi) {
      for (Shard& sd : e->sh) {
        k_pack_rows<<<kPackGrid, 256, 0, s>>>(sd.d_par, T, d2);
        TICK_CHECK("k_pack_rows");
      }
      if (int32_t rc = exchange_counts(e, d2 ? XK_ACK : XK_REQ)) return rc;
    }
    for (Shard& sd : e->sh) {
      if (multi) {
        k_recv_sync<<<256, 256, 0, s>>>(sd.d_par, T, d2);
        TICK_CHECK("k_recv_sync");
        if (e->pull_rows) {
          k_pull_rows<<<kPackGrid, 256, 0, s>>>(sd.d_par, T, d2);
          TICK_CHECK("k_pull_rows");
        }
      }
      // SYNC: an unsharded engine classifies every SYNC inside k_sync_apply with the block witness
      // (fused, no classify launch), a sharded one streams the rows that arrived from other shards
      // in k_sync_classify.  SYNC_ACK: an unsharded engine classifies its acks inside k_sync_apply
      // (every ack is local, and almost all reuse the SYNC merge's reverse classification); a sharded
      // one streams the acks that arrived with their rows from other shards
      const int fused = !multi && d2 == 0;
      const int classified = (d2 == 0 && !fused) || multi;
      if (classified) launch_classify(e, sd, d2);
      TICK_CHECK("k_sync_classify");
      launch_apply(e, sd, d2, classified, fused);
      TICK_CHECK(d2 ? "k_ack_apply" : "k_sync_apply");
      if (d2 == 0 && sd.c.delay_on) {  // delayed SYNC_ACKs: contents parked, the acks deferred
        k_ack_delay<<<256, 256, 0, s>>>(sd.d_par, T);
        TICK_CHECK("k_ack_delay");
      }
    }
  }
  for (Shard& sd : e->sh) {
    // ---- end of tick (also zeroes the per-tick counters and applies other shards' stops)
    const uint32_t ge = grid_for(std::max<uint32_t>(sd.c.nl, 64), 256);
    k_end_tick<<<ge, REB_BLOCK, 0, s>>>(sd.d_par, T, (T % kRebaseEvery) == 0 ? 1 : 0);
    TICK_CHECK("k_end_tick");
  }
  return SWIM_OK;
}

// ---- quiet windows (swim_quiet.h).  The host side of the eligibility: nothing the device check does
// not cover may be pending or configured — control operations (joins, address binds), the loss and
// per-link settings of the NetworkEmulator, a partition, message delay, address routes, recorded FD
// events — and the engine is unsharded or a local group.
constexpr uint32_t kQuietMax = 4096;         // ticks per window at most
constexpr uint32_t kQuietBackoffMax = 1024;  // ticks between tries while the cluster is not quiet
// Every input here is replicated control state, identical on every rank of an RCCL engine (all
// control calls are collective), so all ranks take the same decision — the window's collective below
// is entered by all of them or by none.
static bool quiet_eligible(const swim_engine* e) {
  if (!e->quiet_on || !e->joins.empty() || !e->binds.empty() || !e->route_h.empty()) return false;
  if (!e->links_h.empty() || e->loss_nz) return false;
  const Ctx& c = e->sh[0].c;
  return !c.partition && !c.delay_on && !c.record_fd;
}

// the recorded windows' kernel times into qprof_ms (the events are complete once synchronised; the
// runtime may mark them done after the spinning wait saw the work finish)
static void qev_flush(swim_engine* e) {
  for (uint32_t k = 0; k < e->qev_n; ++k) {
    float ms = 0.f;
    hipEventSynchronize(e->qev[2 * k + 1]);
    if (hipEventElapsedTime(&ms, e->qev[2 * k], e->qev[2 * k + 1]) == hipSuccess) e->qprof_ms += ms;
  }
  e->qev_n = 0;
}

// an API call that changes state or configuration: the next quiet window scans again
static inline void mutated(swim_engine* e) {
  if (e) e->pre_valid = false;
}

// One window of up to K ticks from tick T + 1: every shard's scan, then every shard's apply (a local
// group shares one control block), then the window's length is read back.
static int32_t run_quiet(swim_engine* e, uint32_t K, uint32_t* done) {
  hipStream_t s = e->stream;
  const uint64_t T0 = e->T + 1;
  for (Shard& sd : e->sh) {
    sd.c.T = T0;
    sync_params(e, sd);
  }
  QuietCtl* q = e->d_quiet + e->q_par;  // reset by the previous window's apply (or at creation)
  QuietCtl* q_next = e->d_quiet + (e->q_par ^ 1u);
  e->q_par ^= 1u;
  // the previous window's apply found this one's end already (no scan), and precomputes the next.
  // RCCL: each rank's apply precomputed its own rows' end; the window is their minimum (one 8-byte
  // allreduce below instead of the scan and the refs' allreduces — a pristine cluster's refs do not
  // change in a quiet window, so the agreement the last scan established still holds).  pre_on,
  // pristine, pre_valid and the window's bounds are replicated host state: every rank takes the same
  // branch and enters the same collectives.
  const bool pre_ok = e->pre_on && e->pristine;
  const bool use_pre = pre_ok && e->pre_valid && e->pre_T0 == T0 && K <= e->pre_H;
  // (the precompute covers the longest window a call can ask for, so the next call's window, whatever
  // its length, needs no scan: the bench's timed call follows a shorter warmup call)
  const uint32_t H = pre_ok ? kQuietMax : 0u;
  uint64_t* pre_in = e->d_pre + e->pre_slot;
  uint64_t* pre_out = e->d_pre + (e->pre_slot ^ 1u);
  const uint32_t tag_in = e->pre_tag, tag_out = e->pre_tag + 1;
  const bool prof = e->prof && e->qev[0];
  if (prof && e->qev_n == swim_engine::kQevRing) qev_flush(e);
  hipEvent_t* qp = e->qev + 2 * e->qev_n;
  if (prof) hipEventRecord(qp[0], s);
  // the shards' witness refs must agree (k_quiet_scan): RCCL compares the ranks' elementwise min and max
  if (e->rccl && !use_pre) {
    const size_t n = e->n;
    if (!e->d_refmm && hipMalloc((void**)&e->d_refmm, 8 * n) != hipSuccess) return SWIM_ENOMEM;
    if (hipMemcpyAsync(e->d_refmm, e->sh[0].c.ref, 4 * n, hipMemcpyDeviceToDevice, s) != hipSuccess ||
        hipMemcpyAsync(e->d_refmm + n, e->sh[0].c.ref, 4 * n, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return SWIM_EDEVICE;
    if (ncclGroupStart() != ncclSuccess) return SWIM_EDEVICE;
    ncclAllReduce(e->d_refmm, e->d_refmm, n, ncclUint32, ncclMin, e->comm, s);
    ncclAllReduce(e->d_refmm + n, e->d_refmm + n, n, ncclUint32, ncclMax, e->comm, s);
    if (nccl_ok(ncclGroupEnd()) != SWIM_OK) return SWIM_EDEVICE;
  }
  if (e->rccl && use_pre &&
      nccl_ok(ncclAllReduce(pre_in, pre_in, 1, ncclUint64, ncclMin, e->comm, s)) != SWIM_OK)
    return SWIM_EDEVICE;
  if (!use_pre) {
    for (Shard& sd : e->sh) {
      const uint32_t g = std::max<uint32_t>(64, grid_for(sd.c.nl, 256));
      const uint32_t* ra = e->rccl ? e->d_refmm : e->world > 1 ? e->sh[0].c.ref : nullptr;
      const uint32_t* rb = e->rccl ? e->d_refmm + e->n : sd.c.ref;
      k_quiet_scan<<<g, 256, 0, s>>>(sd.d_par, T0, K, q, ra, rb, e->pristine ? 1u : 0u);
    }
    // RCCL: the window is the minimum over the ranks (fail tick, min table size, 0xffffffff - max)
    if (e->rccl && nccl_ok(ncclAllReduce(q, q, 3, ncclUint32, ncclMin, e->comm, s)) != SWIM_OK)
      return SWIM_EDEVICE;
  }
  for (Shard& sd : e->sh) {
    const uint32_t g = std::max<uint32_t>(64, grid_for(sd.c.nl, 256));
    k_quiet_apply<<<g, 256, 0, s>>>(sd.d_par, T0, K, use_pre ? nullptr : q, q_next, e->d_done,
                                    (uint32_t)kRebaseEvery, pre_in, tag_in, pre_out, tag_out, H);
  }
  e->pre_tag = tag_out;
  e->pre_slot ^= 1u;
  if (prof) {
    hipEventRecord(qp[1], s);
    e->qev_n++;
  }
  // (the drain after a window that ends the swim_step call needs no wait of its own.  Publishing the
  // status words from the apply's last workgroup instead of k_status measured slower both ways: with a
  // release fence per workgroup (its XCD's L2 written back) and without (256 workgroups' counter
  // atomics on one address serialise at the L2): 2.0 / 2.6 vs 2.9 x 10^10 member-periods/s)
  if (e->spin_wait) {
    const uint32_t seq = ++e->status_seq;
    launch_status(e, seq);
    if (wait_status_seq(e, seq) != SWIM_OK) return SWIM_EDEVICE;
  } else {
    launch_status(e);
    if (hipStreamSynchronize(s) != hipSuccess) return SWIM_EDEVICE;
  }
  e->par_slot = 0;  // (the stream drained: the Params staging ring restarts)
  *done = std::min(__atomic_load_n(e->h_done, __ATOMIC_ACQUIRE), K);
  if (prof) {
    // algorithmic bytes (swim.h swim_profile_quiet): SURVEY.md §8(d)'s 21 B per member-period of the
    // ping phase, plus what the quiet check must read once per window: every owned row's count of
    // non-zero witness blocks, 64 B of per-member words, the reference row, the window's timer buckets
    uint64_t rows = 0, nq = 0;
    for (const Shard& sd : e->sh) {
      rows += sd.c.nl;
      nq += sd.c.wheel_nq;
    }
    const uint64_t mp = rows * (uint64_t)*done / e->P;
    e->qprof_windows++;
    e->qprof_ticks += *done;
    e->qprof_mp += mp;
    e->qprof_bytes += 21ull * mp + rows * (4ull + 64ull) + 4ull * e->n * e->sh.size() +
                      4ull * std::min<uint64_t>(K, e->sh[0].c.wheel_mask + 1ull) * nq;
  }
  e->T += *done;
  e->host_ticks += *done;
  e->pre_valid = H > 0 && *done > 0;  // (a window cut short is followed by a per-tick tick: cleared)
  e->pre_T0 = e->T + 1;
  e->pre_H = H;
  if (use_pre) e->qst.precomputed++;
  e->qst.attempts++;
  if (*done) {
    e->qst.windows++;
    e->qst.ticks += *done;
  }
  if (*done < K) e->qst.cut_short++;
  return SWIM_OK;
}

static int32_t upload_links(swim_engine* e) {
  auto& L = e->links_h;
  std::sort(L.begin(), L.end(), [](const LinkDev& x, const LinkDev& y) { return x.a < y.a || (x.a == y.a && x.b < y.b); });
  for (Shard& sd : e->sh) {
    if (L.size() > sd.links_dev_cap) {
      uint32_t cap = next_pow2((uint32_t)L.size());
      LinkDev* p = nullptr;
      if (!sd.alloc(&p, cap)) return SWIM_ENOMEM;
      sd.c.links = p;
      sd.links_dev_cap = cap;
    }
    if (!L.empty() && hipMemcpy(sd.c.links, L.data(), sizeof(LinkDev) * L.size(), hipMemcpyHostToDevice) != hipSuccess)
      return SWIM_EDEVICE;
    sd.c.n_links = (uint32_t)L.size();
  }
  return SWIM_OK;
}

static LinkDev* find_link_h(swim_engine* e, uint32_t a, uint32_t b, bool create) {
  for (auto& L : e->links_h)
    if (L.a == a && L.b == b) return &L;
  if (!create) return nullptr;
  e->links_h.push_back(LinkDev{a, b, -1, -1, -1});
  return &e->links_h.back();
}

static void prune_links(swim_engine* e) {
  auto& L = e->links_h;
  L.erase(std::remove_if(L.begin(), L.end(),
                         [](const LinkDev& x) { return x.out_loss < 0 && x.in_pass < 0 && x.out_delay == -1; }),
          L.end());
}

static int32_t read_member_dev(swim_engine* e, Shard& sd, uint32_t m, MemberDev* out) {
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return hipMemcpy(out, sd.c.mem + (m - sd.c.lo), sizeof(MemberDev), hipMemcpyDeviceToHost) == hipSuccess ? SWIM_OK
                                                                                                          : SWIM_EDEVICE;
}
static int32_t write_member_dev(Shard& sd, uint32_t m, const MemberDev& in) {
  return hipMemcpy(sd.c.mem + (m - sd.c.lo), &in, sizeof(MemberDev), hipMemcpyHostToDevice) == hipSuccess ? SWIM_OK
                                                                                                         : SWIM_EDEVICE;
}
static int32_t read_gsched(Shard& sd, uint32_t m, GossipSched* out) {
  return hipMemcpy(out, sd.c.gs + (m - sd.c.lo), sizeof(GossipSched), hipMemcpyDeviceToHost) == hipSuccess ? SWIM_OK
                                                                                                          : SWIM_EDEVICE;
}
static int32_t read_up(swim_engine* e, uint32_t m, uint8_t* up) {
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return hipMemcpy(up, e->sh[0].c.up + m, 1, hipMemcpyDeviceToHost) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
}
// replicated byte array write on every local shard
static int32_t set_replicated(swim_engine* e, size_t field_off, uint32_t m, uint8_t v, bool all) {
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  for (Shard& sd : e->sh) {
    uint8_t* base = *reinterpret_cast<uint8_t**>(reinterpret_cast<char*>(&sd.c) + field_off);
    hipError_t r = all ? hipMemset(base, v, e->n) : hipMemcpy(base + m, &v, 1, hipMemcpyHostToDevice);
    if (r != hipSuccess) return SWIM_EDEVICE;
  }
  return SWIM_OK;
}

// leaveCluster (MembershipProtocolImpl.java:233-242) on the device: LEAVING inc+1, spread gossip
__global__ void k_leave(Ctx c, uint32_t v, int32_t stop_after) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  MemberDev& m = mem(c, v);
  const uint64_t cell = cell_get(c, v, v);
  const int32_t inc = c_inc(cell) + 1;
  cell_put(c, v, v, c_with_record(cell, SWIM_LEAVING, inc));
  spread_gossip(c, v, v, SWIM_LEAVING, inc, SWIM_ORIG_LEAVE);
  if (stop_after) {
    m.leave_pending = 1;
    m.leave_gossiper = v;
    m.leave_seq = m.g_counter - 1;
  }
}

// ClusterImpl.updateMetadata (:497-500) + updateIncarnation (MembershipProtocolImpl.java:214-226)
__global__ void k_update_meta(Ctx c, uint32_t v, int owner) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  c.meta_ver[v]++;
  if (!owner) return;
  const uint64_t cell = cell_get(c, v, v);
  const int32_t inc = c_inc(cell) + 1;
  cell_put(c, v, v, c_with_record(cell, SWIM_ALIVE, inc));
  spread_gossip(c, v, v, SWIM_ALIVE, inc, SWIM_ORIG_METADATA);
}

// swim_ingest_sync: syncMembership (MembershipProtocolImpl.java:491-509) at viewer v over externally
// supplied records, one workgroup: thread 0 runs updateMembership record by record, then the ALIVE
// admissions whose fetch succeeded; the workgroup then applies the pingMembers inserts in event order.
// No REMOVED arises (DEAD records are refused by the host side), so the lists need no compaction.
__global__ void __launch_bounds__(256) k_ingest_sync(Params* P, uint64_t T, uint32_t v, const swim_record* rec,
                                                     uint32_t n, int32_t initial) {
  const Ctx c = pctx_sync(P, T);
  __shared__ uint32_t s_iP[256], s_iS[256], s_iR[256];
  const int reason = initial ? R_INITIAL_SYNC : R_SYNC;
  uint64_t* pend = P->b.pend;  // (workgroup 0's slice of the SYNC apply's pending admissions)
  if (threadIdx.x == 0) {
    MemberDev& m = mem(c, v);
    // the control phase's event minors and fetch draws run on across the operations of one tick
    // (two ingestions between the same ticks: distinct event keys, distinct draws)
    if (m.ctl_tick1 != (uint32_t)T + 1) {
      m.ev_minor = 0;
      m.fetch_ctr = 0;
      m.ctl_tick1 = (uint32_t)T + 1;
    }
    uint32_t npend = 0;
    for (uint32_t i = 0; i < n; ++i)
      if (update_membership(c, v, rec[i].member, rec[i].status, rec[i].inc, reason, SWIM_PHASE_CONTROL))
        pend[npend++] = ((uint64_t)rec[i].member << 32) | (uint32_t)rec[i].inc;
    for (uint32_t j = 0; j < npend; ++j)
      apply_alive(c, v, (uint32_t)(pend[j] >> 32), (int32_t)(uint32_t)pend[j], reason, SWIM_PHASE_CONTROL);
    stat_add(c, ST_SYNC_ACKS, 1);
    stat_add(c, ST_SYNC_RECORDS, n);
  }
  __syncthreads();
  apply_ins_batch<256, true>(c, v, threadIdx.x, s_iP, s_iS, s_iR);
}

__global__ void k_spread(Ctx c, uint32_t v, uint32_t payload) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  spread_user(c, v, payload);
}

// The producer side of a shard's exchange, one region (one IPC handle): tx_msgs, tx_reqs, tx_acks,
// tx_stops, tx_rows[2], at offsets that are the same on every rank.  With RCCL it is uncached, so the
// producers' stores land in HBM, where the peers' system-scope loads over xGMI read them.
struct XLayout {
  size_t o_msgs, o_reqs, o_acks, o_stops, o_rows0, o_rows1, bytes;
};
static XLayout xlayout(const swim_engine* e, const Bufs& b, uint32_t row_cap) {
  const size_t W = (size_t)e->world, rows = (size_t)row_cap * e->n * 4;
  XLayout L{};
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  L.o_msgs = take(W * b.tx_msg_cap * sizeof(GMsgFull));
  L.o_reqs = take(W * b.tx_req_cap * sizeof(SyncReq));
  L.o_acks = take(W * b.tx_req_cap * sizeof(SyncReq));
  L.o_stops = take(4ull * b.tx_stop_cap);
  L.o_rows0 = take(rows);
  L.o_rows1 = take(rows);
  L.bytes = off;
  return L;
}
static size_t xreg_bytes_for(const swim_engine* e, const Bufs& b, uint32_t row_cap) { return xlayout(e, b, row_cap).bytes; }
static void* xreg_alloc(size_t bytes, bool uncached, bool* got_uncached) {
  void* p = nullptr;
  hipError_t r = hipErrorUnknown;
  if (uncached) r = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
  if (got_uncached) *got_uncached = r == hipSuccess;
  if (r != hipSuccess) r = hipMalloc(&p, bytes);
  return r == hipSuccess ? p : nullptr;
}
// the shard's exchange region becomes `fresh` (sized for row_cap): everything before the rows —
// message and SYNC headers, stops, deferred acks — keeps its offset and is carried over; the old
// region is freed
static int32_t xreg_install(swim_engine* e, Shard& sd, void* fresh, uint32_t row_cap) {
  Bufs& b = sd.b;
  const XLayout L = xlayout(e, b, row_cap);
  void* old = sd.xreg;
  if (old) {
    const size_t keep = std::min(L.o_rows0, sd.xreg_bytes);
    if (keep && hipMemcpy(fresh, old, keep, hipMemcpyDeviceToDevice) != hipSuccess) return SWIM_EDEVICE;
    hipFree(old);
  }
  sd.xreg = fresh;
  sd.xreg_bytes = L.bytes;
  b.row_cap = row_cap;
  char* base = static_cast<char*>(fresh);
  b.tx_msgs = reinterpret_cast<GMsgFull*>(base + L.o_msgs);
  b.tx_reqs = reinterpret_cast<SyncReq*>(base + L.o_reqs);
  b.tx_acks = reinterpret_cast<SyncReq*>(base + L.o_acks);
  b.tx_stops = reinterpret_cast<uint32_t*>(base + L.o_stops);
  b.tx_rows[0] = reinterpret_cast<uint32_t*>(base + L.o_rows0);
  b.tx_rows[1] = reinterpret_cast<uint32_t*>(base + L.o_rows1);
  return SWIM_OK;
}
// (re)allocates the shard's exchange region for its row_cap; on failure the old region stays
static int32_t alloc_xreg(swim_engine* e, Shard& sd, bool uncached) {
  bool unc = false;
  void* fresh = xreg_alloc(xreg_bytes_for(e, sd.b, sd.b.row_cap), uncached, &unc);
  if (!fresh) return SWIM_ENOMEM;
  if (int32_t rc = xreg_install(e, sd, fresh, sd.b.row_cap)) {
    hipFree(fresh);
    return rc;
  }
  sd.xreg_uncached = unc;
  return SWIM_OK;
}

static int32_t alloc_shard(swim_engine* e, Shard& sd, uint32_t shard, uint32_t n_initial, uint64_t seed) {
  const swim_config& cf = e->cfg;
  Ctx& c = sd.c;
  Bufs& b = sd.b;
  const uint32_t n = e->n;
  c.n = n;
  c.sz = e->sz;
  c.rank = shard;
  c.world = (uint32_t)e->world;
  c.xchg = e->xchg ? 1u : 0u;
  c.lo = std::min(n, shard * e->sz);
  c.nl = std::min(n, c.lo + e->sz) - c.lo;
  const uint32_t nl = c.nl;
  c.gcap = next_pow2(cf.gossip_capacity ? cf.gossip_capacity : 1024);  // (a power of two: the slab is a ring)
  c.hcap = next_pow2(cf.collector_capacity ? cf.collector_capacity : 4096);
  c.gix_mask = next_pow2(2 * c.gcap) - 1;
  // infected overflows a member holds at once: states that took a second sender after a collector
  // clear (segmentation), an eighth of the slab (32 B each: +1/6 of the slab's bytes).  Config 3's
  // churn clears collectors every period: more than 4,096 live at N = 16,384 by its fourth period
  c.inf_mask = next_pow2(std::max<uint32_t>(64, c.gcap / 8)) - 1;
  // spilled collectors by tier (6 / 62 / 510 / 16,382 intervals); blocks are recycled, so these
  // bound the collectors spilled at once, not over the run
  const uint64_t icap = cf.interval_capacity ? cf.interval_capacity : 64;  // tier-0 blocks per row
  const uint64_t rows = std::max(nl, 1u);
  c.spill_cap[0] = (uint32_t)std::min<uint64_t>(1ull << 31, std::max<uint64_t>(1u << 18, icap * rows));
  c.spill_cap[1] = (uint32_t)std::min<uint64_t>(1ull << 30, std::max<uint64_t>(1u << 15, icap * rows / 8));
  c.spill_cap[2] = (uint32_t)std::min<uint64_t>(1ull << 28, std::max<uint64_t>(1u << 12, icap * rows / 128));
  c.spill_cap[3] = (uint32_t)std::min<uint64_t>(1ull << 26, std::max<uint64_t>(1u << 10, icap * rows / 1024));
  c.P = e->P;
  c.to_ticks = (uint32_t)cf.ping_timeout / e->tick_ms;
  c.relay_ticks = e->P - c.to_ticks;
  c.G = e->G;
  c.S = e->S;
  c.sync_to_ticks = (uint32_t)cf.sync_timeout / e->tick_ms;
  c.metadata_timeout = (uint32_t)cf.metadata_timeout;
  c.tick_ms = e->tick_ms;
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
  const uint64_t tcap = cf.timer_capacity ? cf.timer_capacity : 2ull * std::max(nl, 1u);
  c.wheel_nq = std::max(1u, (nl + 255) / 256);  // one queue per k_fd workgroup
  // paged wheel (swim_device.h): one (bucket, queue) may take 2x its block's even share of the
  // per-tick capacity (timers cluster on viewers unevenly: a churn tick schedules ~16 timers at each
  // of 256 viewers of a block), at most every (viewer, subject) pair of the block; its page table has
  // ~1,024 pages (the page grows from 64 to 4,096 entries with that bound); the pool holds
  // timer_pool_capacity entries in whole pages plus one partial page per (bucket, queue)
  {
    const uint64_t W = (uint64_t)c.wheel_mask + 1, nq = c.wheel_nq;
    const uint64_t per_q = std::min<uint64_t>(256ull * n, std::max<uint64_t>(4096, 2 * ((tcap + nq - 1) / nq)));
    uint32_t sh = 6;
    while (sh < 12 && (per_q >> sh) > 1024) ++sh;
    c.wheel_pshift = sh;
    c.wheel_ptmax = (uint32_t)((per_q + (1ull << sh) - 1) >> sh);
    const uint64_t pool = cf.timer_pool_capacity ? cf.timer_pool_capacity : std::min<uint64_t>(1ull << 27, W * tcap);
    c.wheel_pages = (uint32_t)std::min<uint64_t>(1ull << 30, ((pool + (1ull << sh) - 1) >> sh) + W * nq + 64);
  }
  c.ev_cap = std::max<uint32_t>(1024, (cf.event_capacity ? cf.event_capacity : (1u << 22)) / SUBQ);
  // deferred pingMembers inserts of one phase: a join burst adds every joiner at every viewer
  c.ins_cap = (uint32_t)std::min<uint64_t>(1ull << 28, std::max<uint64_t>(1ull << 22, 256ull * nl));
  // a sharded engine's inboxes hold 4x as many per receiver: a GOSSIP_REQ from another shard is
  // materialised even when the receiver already holds its gossip (k_recv_msgs flags it; the emitter
  // could not read this shard's receipt bits): the failures storm at N = 65,536 sends ~1,500 a round
  // per receiver
  b.msg_cap = cf.message_capacity ? cf.message_capacity
                                 : (uint32_t)std::min<uint64_t>(1ull << 28, std::max<uint64_t>(
                                                                    1ull << 20, (e->xchg ? 2048ull : 512ull) * nl));
  // inbox pages: the message capacity in 64-message pages plus one partial page per receiver; one
  // receiver's inbox may span pg_max pages: 64x its even share of the capacity, at least 512 pages
  // (32 Ki messages: a storm's inboxes are uneven), at most the whole pool
  // (+ nl: every receiver's own first page, inbox_page_alloc)
  b.pg_cap = (uint32_t)std::min<uint64_t>(1ull << 26, (uint64_t)b.msg_cap / 64 + 2ull * nl + 64);
  b.pg_max = (uint32_t)std::min<uint64_t>(b.pg_cap, std::max<uint64_t>(512, next_pow2((uint32_t)std::min<uint64_t>(
                                              1u << 30, 64ull * b.msg_cap / 64 / std::max(nl, 1u)))));
  b.pg_max = std::min<uint32_t>(b.pg_max, 1u << 14);
  b.req_cap = std::max<uint32_t>(1u << 12, 4 * n);
  b.wave_min = cf.deliver_wave_min ? std::min<uint32_t>(cf.deliver_wave_min, DLV_SORT) : (uint32_t)DLV_SORT;
  b.coop_min = COOP_MIN;
  if (const char* cm = std::getenv("SWIM_DEBUG_COOP_MIN"))  // tests: the whole-wave path for small inboxes too
    if (std::atoi(cm) > 0) b.coop_min = (uint32_t)std::atoi(cm);
  b.dq_bcap = 0;  // the delay ring is allocated when a delay is first set (swim_set_*_delay)
  // snapshot rows for members that both send and receive a SYNC in one tick (at most two each: the
  // SYNC content and, when its merges changed the row, the SYNC_ACK content): a few per tick in
  // steady state, up to every member right after a partition heals; at most 1 GiB of rows
  b.snap_cap = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2ull * nl, std::max<uint64_t>(256, (1ull << 28) / std::max(n, 1u))));
  b.sy_max = (SY_INBOX - SY_INLINE + 63) / 64;
  b.sy_pool_cap = b.req_cap / 64 + std::min(nl, b.req_cap) + 64;
  b.chunks = (n + SYNC_CHUNK - 1) / SYNC_CHUNK;
  b.pool_cap = std::max<uint32_t>(1u << 22, 16 * n);
  const bool multi = e->xchg;
  // tx capacities must be identical on every rank: both ends of a send clamp the count with them
  // (the failures storm at N = 65,536 over 2 shards sends ~24 M GOSSIP_REQs a round to the peer;
  // all peers' buffers together: 32 KiB per member of the whole cluster, 2 GiB at N = 65,536)
  // (an explicit message_capacity — a shard's inbox — also sizes each destination's share of the
  // outgoing buffer: message_capacity / world, when that is larger)
  b.tx_msg_cap = multi ? (uint32_t)std::min<uint64_t>(1ull << 28, std::max<uint64_t>({1ull << 20, 1024ull * e->sz,
                                                                                  (uint64_t)cf.message_capacity / (uint64_t)e->world}))
                       : 0;
  b.tx_req_cap = multi ? b.req_cap : 0;
  b.tx_stop_cap = multi ? kStopCap : 0;
  // content rows one shard may send in one SYNC (or SYNC_ACK) exchange: 256 MiB of rows, 64..4,096
  b.row_cap = multi ? std::min<uint32_t>(4096, std::max<uint32_t>(64, (1u << 26) / std::max(n, 1u))) : 0;
  if (const char* rc = std::getenv("SWIM_DEBUG_ROW_CAP"))  // tests: start small so that joins grow it
    if (multi && std::atoi(rc) > 0) b.row_cap = (uint32_t)std::atoi(rc);

  const size_t nn = (size_t)nl * n;
  c.blocks = (n + (1u << BLK_SHIFT) - 1) >> BLK_SHIFT;
  bool ok = sd.alloc(&c.recs, nn) && sd.alloc(&c.aux, nn) && sd.alloc(&c.ref, n) && sd.alloc(&c.dirty, n) &&
            sd.alloc(&c.bdiff, (size_t)std::max(nl, 1u) * c.blocks) && sd.alloc(&c.bnz, std::max(nl, 1u)) && sd.alloc(&c.mem, nl) && sd.alloc(&c.up, n) && sd.alloc(&c.ping, nn) &&
            sd.alloc(&c.remote, nn) && sd.alloc(&c.slab_hot, (size_t)nl * c.gcap) && sd.alloc(&c.slab_cold, (size_t)nl * c.gcap) &&
            sd.alloc(&c.inf_over, (size_t)std::max(nl, 1u) * (c.inf_mask + 1)) &&
            sd.alloc(&c.gix, (size_t)nl * (c.gix_mask + 1)) && sd.alloc(&c.coll, (size_t)nl * c.hcap) &&
            sd.alloc(&c.spill[0], (size_t)c.spill_cap[0] * tier_words(0)) &&
            sd.alloc(&c.spill[1], (size_t)c.spill_cap[1] * tier_words(1)) &&
            sd.alloc(&c.spill[2], (size_t)c.spill_cap[2] * tier_words(2)) &&
            sd.alloc(&c.spill[3], (size_t)c.spill_cap[3] * tier_words(3)) &&
            sd.alloc(&c.spill_avail[0], c.spill_cap[0]) && sd.alloc(&c.spill_freed[0], c.spill_cap[0]) &&
            sd.alloc(&c.spill_avail[1], c.spill_cap[1]) && sd.alloc(&c.spill_freed[1], c.spill_cap[1]) &&
            sd.alloc(&c.spill_avail[2], c.spill_cap[2]) && sd.alloc(&c.spill_freed[2], c.spill_cap[2]) &&
            sd.alloc(&c.spill_avail[3], c.spill_cap[3]) && sd.alloc(&c.spill_freed[3], c.spill_cap[3]) &&
            sd.alloc(&c.spill_ctl, NTIER) && sd.alloc(&c.seg_flag, nl) &&
            sd.alloc(&c.fd_sync, (size_t)nl * FD_SYNC_MAX) &&
            sd.alloc(&c.wheel, (size_t)c.wheel_pages << c.wheel_pshift) &&
            sd.alloc(&c.wheel_cnt, (size_t)(c.wheel_mask + 1) * c.wheel_nq) &&
            sd.alloc(&c.wheel_pt, (size_t)(c.wheel_mask + 1) * c.wheel_nq * c.wheel_ptmax) &&
            sd.alloc(&c.wheel_avail, c.wheel_pages) && sd.alloc(&c.wheel_freed, c.wheel_pages) &&
            sd.alloc(&c.wheel_ctl, 1) && sd.alloc(&c.ev, (size_t)c.ev_cap * SUBQ) &&
            sd.alloc(&c.ev_cnt, SUBQ) && sd.alloc(&c.default_loss, n) &&
            sd.alloc(&c.default_delay, n) && sd.alloc(&b.dq_cnt, DQ_BUCKETS) && sd.alloc(&c.meta_ver, n) &&
            sd.alloc(&c.default_inbound, n) && sd.alloc(&c.group, n) && sd.alloc(&c.links, 1) &&
            sd.alloc(&c.is_seed, n) && sd.alloc(&c.seeds, n) && sd.alloc(&c.ins, c.ins_cap) &&
            sd.alloc(&c.ins_inline, (size_t)nl * INS_INLINE) && sd.alloc(&c.compact_flag, nl) &&
            sd.alloc(&c.fd_next, nl) && sd.alloc(&c.sync_next, nl) && sd.alloc(&c.mflag, nl) &&
            sd.alloc(&c.gs, std::max(nl, 1u)) &&
            sd.alloc(&c.gslot, GSLOTS) && sd.alloc(&c.gpend, GSLOTS) &&
            sd.alloc(&c.gbits, (size_t)std::max(nl, 1u) * GROW) && sd.alloc(&c.clr_tick, std::max(nl, 1u)) &&
            sd.alloc(&c.gclaim, 2 * GSLOTS) && sd.alloc(&c.gclaim_cnt, 2) &&
            sd.alloc(&c.stats, (size_t)ST_COUNT * ST_REPL) && sd.alloc(&c.err, 1) && sd.alloc(&sd.k, 1) &&
            sd.alloc(&sd.x, 1) && sd.alloc(&b.pg_msgs, (size_t)b.pg_cap * 64) &&
            sd.alloc(&b.pg_perm, (size_t)b.pg_cap * 64) && sd.alloc(&b.pg_tab, (size_t)std::max(nl, 1u) * b.pg_max) &&
            sd.alloc(&b.msg_cnt, nl) && sd.alloc(&b.big_list, nl) && sd.alloc(&b.big_tick, nl) &&
            sd.alloc(&b.reqs, b.req_cap) && sd.alloc(&b.req_cnt, nl) && sd.alloc(&b.req_recv, nl) &&
            sd.alloc(&b.acks, b.req_cap) && sd.alloc(&b.ack_cnt, nl) &&
            sd.alloc(&b.rq_inl, (size_t)std::max(nl, 1u) * SY_INLINE) && sd.alloc(&b.ack_inl, (size_t)std::max(nl, 1u) * SY_INLINE) &&
            sd.alloc(&b.rq_tab, (size_t)std::max(nl, 1u) * b.sy_max) && sd.alloc(&b.rq_pool, (size_t)b.sy_pool_cap * 64) &&
            sd.alloc(&b.ack_tab, (size_t)std::max(nl, 1u) * b.sy_max) && sd.alloc(&b.ack_pool, (size_t)b.sy_pool_cap * 64) &&
            sd.alloc(&b.ack_snap, nl) && sd.alloc(&b.snap_ready, nl) && sd.alloc(&b.sflag, nl) &&
            sd.alloc(&b.ack_chunk, (size_t)b.req_cap * b.chunks) && sd.alloc(&b.ack_ctot, b.req_cap) &&
            sd.alloc(&b.ack_recv, nl) && 
            sd.alloc(&b.snap, (size_t)b.snap_cap * (n + c.blocks)) && sd.alloc(&b.snap_idx, nl) &&
            sd.alloc(&b.snap_list, 2 * (size_t)b.snap_cap) && sd.alloc(&b.snap_cnt, 2) && sd.alloc(&b.item_chunk, (size_t)b.req_cap * b.chunks) &&
            sd.alloc(&b.item_total, b.req_cap) && sd.alloc(&b.pool, b.pool_cap) &&
            sd.alloc(&b.rev_chunk, (size_t)b.req_cap * b.chunks) && sd.alloc(&b.rev_total, b.req_cap) &&
            sd.alloc(&b.row_mod, nl) &&
            sd.alloc(&b.pend, (size_t)kApplyGrid * n) && sd.alloc(&sd.d_par, 1) && sd.alloc(&b.senders, nl) &&
            sd.alloc(&c.pa, (size_t)std::max(nl, 1u) * PA_CAP) && sd.alloc(&c.pa_n, std::max(nl, 1u));
  if (ok && multi) {
    ok = alloc_xreg(e, sd, e->rccl) == SWIM_OK && sd.alloc(&b.rx_cnt, 4 * MAXW) &&
         sd.alloc(&b.rx_stops, (size_t)e->world * b.tx_stop_cap) && sd.alloc(&b.rx_stop_n, 1) && sd.alloc(&sd.peers, 1);
    b.peers = sd.peers;
  }
  if (!ok) return SWIM_ENOMEM;
  sd.links_dev_cap = 1;
  c.ins_total = &sd.k->ins_total;
  b.k = sd.k;
  b.x = sd.x;
  hipStream_t s = e->stream;
  hipMemsetAsync(c.coll, 0, sizeof(CollEnt) * (size_t)nl * c.hcap, s);
  hipMemsetAsync(c.inf_over, 0xff, sizeof(InfOver) * (size_t)std::max(nl, 1u) * (c.inf_mask + 1), s);  // INF_EMPTY
  hipMemsetAsync(c.spill_ctl, 0, sizeof(SpillCtl) * NTIER, s);
  hipMemsetAsync(c.seg_flag, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(c.pa_n, 0, 4 * (size_t)std::max(nl, 1u), s);
  c.pa_cap = PA_CAP;
  hipMemsetAsync(c.wheel, 0xff, sizeof(uint64_t) * ((size_t)c.wheel_pages << c.wheel_pshift), s);  // WHEEL_EMPTY
  hipMemsetAsync(c.wheel_cnt, 0, sizeof(uint32_t) * (c.wheel_mask + 1) * c.wheel_nq, s);
  hipMemsetAsync(c.wheel_pt, 0xff, sizeof(uint32_t) * (c.wheel_mask + 1) * c.wheel_nq * c.wheel_ptmax, s);
  hipMemsetAsync(c.wheel_ctl, 0, sizeof(SpillCtl), s);
  hipMemsetAsync(c.ev_cnt, 0, 4 * SUBQ, s);
  hipMemsetAsync(c.up, 0, n, s);
  hipMemsetAsync(c.up, 1, n_initial, s);
  hipMemsetAsync(c.ref, 0, 4 * (size_t)n, s);
  hipMemsetAsync(c.dirty, 0, 4 * (size_t)n, s);
  hipMemsetAsync(c.default_loss, 0, n, s);
  hipMemsetAsync(c.default_delay, 0xff, 2ull * n, s);  // -1: no delay
  hipMemsetAsync(b.dq_cnt, 0, 4ull * DQ_BUCKETS, s);
  c.delay_th = nullptr;
  c.delay_on = 0;
  hipMemsetAsync(c.meta_ver, 0, 4ull * n, s);
  c.meta_seen = nullptr;
  c.ns = nullptr;
  c.ns_rel = nullptr;
  c.n_ns = 0;
  hipMemsetAsync(c.default_inbound, 1, n, s);
  hipMemsetAsync(c.group, 0, 2 * (size_t)n, s);
  hipMemsetAsync(c.is_seed, 0, n, s);
  hipMemsetAsync(c.compact_flag, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(c.gslot, 0, sizeof(GSlot) * GSLOTS, s);
  hipMemsetAsync(c.gpend, 0, sizeof(uint64_t) * GSLOTS, s);
  hipMemsetAsync(c.gbits, 0, sizeof(uint32_t) * GROW * (size_t)std::max(nl, 1u), s);
  hipMemsetAsync(c.clr_tick, 0, sizeof(uint32_t) * std::max(nl, 1u), s);
  hipMemsetAsync(c.gclaim_cnt, 0, sizeof(uint32_t) * 2, s);
  hipMemsetAsync(c.stats, 0, 8 * (size_t)ST_COUNT * ST_REPL, s);
  hipMemsetAsync(c.err, 0, 4, s);
  hipMemsetAsync(sd.k, 0, sizeof(Counters), s);
  hipMemsetAsync(sd.x, 0, sizeof(Xc), s);
  if (multi) {
    hipMemsetAsync(b.rx_cnt, 0, 4 * MAXW * sizeof(uint32_t), s);
    hipMemsetAsync(b.rx_stop_n, 0, sizeof(uint32_t), s);
  }
  hipMemsetAsync(b.msg_cnt, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(b.pg_tab, 0xff, 4 * (size_t)std::max(nl, 1u) * b.pg_max, s);
  {  // every receiver's first inbox page is its own: pg_tab[i][0] = i
    std::vector<uint32_t> own(std::max(nl, 1u));
    for (uint32_t x = 0; x < own.size(); ++x) own[x] = x;
    if (hipMemcpy2DAsync(b.pg_tab, 4ull * b.pg_max, own.data(), 4, 4, own.size(), hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return SWIM_EDEVICE;
  }
  hipMemsetAsync(b.big_tick, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(b.req_cnt, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(b.ack_cnt, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(b.snap_idx, 0xff, 4 * (size_t)nl, s);
  hipMemsetAsync(b.ack_snap, 0xff, 4 * (size_t)nl, s);
  hipMemsetAsync(b.snap_ready, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(b.sflag, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(b.rq_tab, 0xff, 4 * (size_t)std::max(nl, 1u) * b.sy_max, s);
  hipMemsetAsync(b.ack_tab, 0xff, 4 * (size_t)std::max(nl, 1u) * b.sy_max, s);
  hipMemsetAsync(b.row_mod, 0, 4 * (size_t)nl, s);
  hipMemsetAsync(b.snap_cnt, 0, 8, s);
  c.T = 0;
  if (nl) {
    k_init_rows<<<std::min<uint32_t>(nl, 65535), 256, 0, s>>>(c, n_initial);
    k_init_members<<<grid_for(nl, 64), 64, 0, s>>>(c, n_initial, cf.sync_stagger, cf.timer_stagger);
  }
  return SWIM_OK;
}

// offsets of the producer buffers inside a shard's exchange region (identical on every rank)
static size_t xoff(const Shard& sd, const void* p) {
  return (size_t)(static_cast<const char*>(p) - static_cast<const char*>(sd.xreg));
}

// A local group: every shard reads the other shards' buffers directly.  With SWIM_EXCHANGE_PULL=1
// the content rows take the RCCL route instead — pulled by k_pull_rows into per-shard copies — so
// the single-GPU parity tests cover that kernel and its system-scope loads too.
static int32_t setup_peers_local(swim_engine* e) {
  for (Shard& sd : e->sh) {
    Peers ph{};
    const bool stale = sd.rx_row_cap != sd.b.row_cap;  // (both copies are sized together)
    if (e->pull_rows)
      for (int k = 0; k < 2; ++k) {
        if (!sd.rx_rows_h[k] || stale) {
          sd.release(sd.rx_rows_h[k]);
          sd.rx_rows_h[k] = nullptr;
          uint32_t* q = nullptr;
          if (!sd.alloc(&q, (size_t)e->world * sd.b.row_cap * e->n)) return SWIM_ENOMEM;
          sd.rx_rows_h[k] = q;
          sd.rx_row_cap = sd.b.row_cap;
        }
        ph.rx_rows[k] = static_cast<uint32_t*>(sd.rx_rows_h[k]);
      }
    for (uint32_t p = 0; p < (uint32_t)e->world; ++p) {
      const Bufs& pb = e->sh[p].b;
      ph.msgs[p] = pb.tx_msgs;
      ph.hdr[0][p] = pb.tx_reqs;
      ph.hdr[1][p] = pb.tx_acks;
      ph.stops[p] = pb.tx_stops;
      for (int k = 0; k < 2; ++k) {
        ph.rows[k][p] = pb.tx_rows[k];
        ph.rows_in[k][p] = e->pull_rows ? ph.rx_rows[k] + (size_t)p * sd.b.row_cap * e->n : pb.tx_rows[k];
      }
      ph.x[p] = e->sh[p].x;
      // the cross-shard receipt filter (emit): peer p's receipt slots, bits and clear ticks
      const Ctx& pc = e->sh[p].c;
      ph.gslot[p] = pc.gslot;
      ph.gbits[p] = pc.gbits;
      ph.clr_tick[p] = pc.clr_tick;
    }
    if (hipMemcpy(sd.peers, &ph, sizeof ph, hipMemcpyHostToDevice) != hipSuccess) return SWIM_EDEVICE;
    sd.b.rfilter = e->rfilter_on ? 1u : 0u;
  }
  return SWIM_OK;
}

// RCCL: every rank maps the other ranks' exchange regions (IPC handles gathered with ncclAllGather)
// and pulls what they produced for it into rx_rows over xGMI (k_pull_rows).
static int32_t setup_peers_rccl(swim_engine* e) {
  Shard& sd = e->sh[0];
  const uint32_t W = (uint32_t)e->world, me = (uint32_t)e->rank;
  hipIpcMemHandle_t mine;
  if (hipIpcGetMemHandle(&mine, sd.xreg) != hipSuccess) {
    // no handle for an uncached allocation: an ordinary one (the consumers' loads are system-scope)
    if (alloc_xreg(e, sd, false) != SWIM_OK) return SWIM_ENOMEM;
    if (hipIpcGetMemHandle(&mine, sd.xreg) != hipSuccess) return SWIM_EDEVICE;
    e->xflags |= SWIM_XCHG_IPC_FALLBACK;
    std::fprintf(stderr, "libswimgpu: rank %d: exchange region is cached (no IPC handle for uncached memory)\n", e->rank);
  }
  e->xflags |= SWIM_XCHG_IPC;
  uint8_t* d_h = nullptr;
  if (hipMalloc((void**)&d_h, sizeof(hipIpcMemHandle_t) * (W + 1)) != hipSuccess) return SWIM_ENOMEM;
  std::vector<hipIpcMemHandle_t> all(W);
  int32_t rc = SWIM_OK;
  if (hipMemcpy(d_h + sizeof(hipIpcMemHandle_t) * W, &mine, sizeof mine, hipMemcpyHostToDevice) != hipSuccess ||
      nccl_ok(ncclAllGather(d_h + sizeof(hipIpcMemHandle_t) * W, d_h, sizeof(hipIpcMemHandle_t), ncclUint8, e->comm,
                            e->stream)) != SWIM_OK ||
      hipStreamSynchronize(e->stream) != hipSuccess ||
      hipMemcpy(all.data(), d_h, sizeof(hipIpcMemHandle_t) * W, hipMemcpyDeviceToHost) != hipSuccess)
    rc = SWIM_EDEVICE;
  hipFree(d_h);
  if (rc) return rc;
  Peers ph{};
  const bool stale = sd.rx_row_cap != sd.b.row_cap;  // (both copies are sized together)
  for (int k = 0; k < 2; ++k) {  // (grow_rows_for_joins allocates them before the switch)
    if (!sd.rx_rows_h[k] || stale) {
      sd.release(sd.rx_rows_h[k]);
      sd.rx_rows_h[k] = nullptr;
      uint32_t* q = nullptr;
      if (!sd.alloc(&q, (size_t)W * sd.b.row_cap * e->n)) return SWIM_ENOMEM;
      sd.rx_rows_h[k] = q;
      sd.rx_row_cap = sd.b.row_cap;
    }
    ph.rx_rows[k] = static_cast<uint32_t*>(sd.rx_rows_h[k]);
  }
  for (uint32_t p = 0; p < W; ++p) {
    char* base = static_cast<char*>(sd.xreg);
    if (p != me) {
      void* q = nullptr;
      if (hipIpcOpenMemHandle(&q, all[p], hipIpcMemLazyEnablePeerAccess) != hipSuccess) return SWIM_EDEVICE;
      sd.ipc_open.push_back(q);
      base = static_cast<char*>(q);
    }
    ph.msgs[p] = reinterpret_cast<const GMsgFull*>(base + xoff(sd, sd.b.tx_msgs));
    ph.hdr[0][p] = reinterpret_cast<const SyncReq*>(base + xoff(sd, sd.b.tx_reqs));
    ph.hdr[1][p] = reinterpret_cast<const SyncReq*>(base + xoff(sd, sd.b.tx_acks));
    ph.stops[p] = reinterpret_cast<const uint32_t*>(base + xoff(sd, sd.b.tx_stops));
    for (int k = 0; k < 2; ++k) {
      ph.rows[k][p] = reinterpret_cast<const uint32_t*>(base + xoff(sd, sd.b.tx_rows[k]));
      ph.rows_in[k][p] = ph.rx_rows[k] + (size_t)p * sd.b.row_cap * e->n;
    }
    ph.x[p] = nullptr;
  }
  return hipMemcpy(sd.peers, &ph, sizeof ph, hipMemcpyHostToDevice) == hipSuccess ? SWIM_OK : SWIM_EDEVICE;
}

static int32_t create_engine(const swim_config* cfg, uint32_t capacity, uint32_t n_initial, uint64_t seed, int32_t rank,
                             int32_t world, bool rccl, const uint8_t* comm_id, swim_engine** out) {
  if (!cfg || !out || capacity < 2 || n_initial > capacity || capacity > (1u << 24)) return SWIM_EINVAL;
  const swim_config& cf = *cfg;
  if (cf.ping_interval <= 0 || cf.ping_timeout <= 0 || cf.ping_timeout >= cf.ping_interval || cf.gossip_interval <= 0 ||
      cf.sync_interval <= 0 || cf.sync_timeout <= 0 || cf.metadata_timeout <= 0 || cf.suspicion_mult <= 0 ||
      cf.gossip_fanout <= 0 || cf.gossip_fanout > 16 || cf.ping_req_members > 16 || cf.gossip_repeat_mult <= 0)
    return SWIM_EINVAL;
  if (world < 1 || world > MAXW || rank < 0 || rank >= world || (uint32_t)world > capacity) return SWIM_EINVAL;
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
  {
    const char* d = std::getenv("SWIM_DEBUG_SYNC");
    e->debug_sync = d && (d[0] == '1' || d[0] == '2') ? d[0] - '0' : 0;
  }
  e->device = cf.device;
  e->n = capacity;
  e->tick_ms = tick;
  e->P = (uint32_t)cf.ping_interval / tick;
  e->G = (uint32_t)cf.gossip_interval / tick;
  e->S = (uint32_t)cf.sync_interval / tick;
  e->rank = rank;
  e->world = world;
  e->rccl = rccl;
  e->xchg = world > 1 || rccl;
  {
    const char* p = std::getenv("SWIM_EXCHANGE_PULL");
    e->pull_rows = rccl || (p && p[0] == '1');
    // the cross-shard receipt filter: a local group's emit reads the other shards' receipt bits in
    // place (SWIM_RFILTER=0 turns it off: every GOSSIP_REQ to another shard is materialised and the
    // receiver flags the duplicates, as over RCCL, whose peers' bitmaps are not mapped)
    const char* rf = std::getenv("SWIM_RFILTER");
    e->rfilter_on = !rccl && world > 1 && !(rf && rf[0] == '0');
  }
  e->sz = (capacity + (uint32_t)world - 1) / (uint32_t)world;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) { delete e; return SWIM_EDEVICE; }
  e->sh.resize(rccl ? 1 : (size_t)world);
  for (size_t i = 0; i < e->sh.size(); ++i) {
    int32_t rc = alloc_shard(e, e->sh[i], rccl ? (uint32_t)rank : (uint32_t)i, n_initial, seed);
    if (rc != SWIM_OK) { delete e; return rc; }
  }
  if (hipHostMalloc((void**)&e->h_par, sizeof(Params) * kParRing) != hipSuccess) { delete e; return SWIM_ENOMEM; }
  if (hipHostMalloc((void**)&e->h_done, 64, hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&e->d_done, e->h_done, 0) != hipSuccess ||
      hipHostMalloc((void**)&e->h_stat, 4 * (SUBQ + 1) * e->sh.size(), hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&e->d_stat, e->h_stat, 0) != hipSuccess ||
      hipMalloc((void**)&e->d_quiet, 2 * sizeof(QuietCtl)) != hipSuccess ||
      hipMemset(e->d_quiet, 0xff, 2 * sizeof(QuietCtl)) != hipSuccess ||  // both blocks reset: no fail, no sizes
      hipMalloc((void**)&e->d_pre, 2 * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(e->d_pre, 0xff, 2 * sizeof(uint64_t)) != hipSuccess) {
    delete e;
    return SWIM_ENOMEM;
  }
  std::memset(e->h_done, 0, 64);  // (status_seq starts at 0: no stale sequence number)
  {
    const char* q = std::getenv("SWIM_QUIET");
    e->quiet_on = !(q && q[0] == '0');
    const char* sp = std::getenv("SWIM_SPIN");
    e->spin_wait = !(sp && sp[0] == '0');
    const char* qp = std::getenv("SWIM_QUIET_PRE");
    e->pre_on = !(qp && qp[0] == '0');
  }
  e->loss_h.assign(capacity, 0);
  if (e->xchg) {
    if (hipMalloc((void**)&e->d_cnt, sizeof(uint32_t) * 2) != hipSuccess) {
      delete e;
      return SWIM_ENOMEM;
    }
  }
  if (hipStreamSynchronize(e->stream) != hipSuccess || hip_status() != SWIM_OK) { delete e; return SWIM_EDEVICE; }
  if (rccl) {
    ncclUniqueId id;
    std::memcpy(&id, comm_id, sizeof(id));
    if (nccl_ok(ncclCommInitRank(&e->comm, world, id, rank)) != SWIM_OK) { delete e; return SWIM_EDEVICE; }
  }
  if (e->xchg) {
    const int32_t rc = rccl ? setup_peers_rccl(e) : setup_peers_local(e);
    if (rc != SWIM_OK) { delete e; return rc; }
  }
  e->g_residue.assign(e->G, cf.timer_stagger ? 1 : 0);  // staggered gossip timers use every residue
  e->g_residue[0] = 1;
  e->is_seed_h.assign(capacity, 0);
  e->joined_h.assign(capacity, 0);
  std::fill(e->joined_h.begin(), e->joined_h.begin() + n_initial, 1);
  e->join_pending_h.assign(capacity, 0);
  *out = e;
  return SWIM_OK;
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
  if (!cfg) return SWIM_EINVAL;
  const int32_t shards = cfg->local_shards > 1 ? cfg->local_shards : 1;
  return create_engine(cfg, capacity, n_initial, seed, 0, shards, false, nullptr, out);
}

int32_t swim_comm_unique_id(uint8_t* out) {
  if (!out) return SWIM_EINVAL;
  ncclUniqueId id;
  if (nccl_ok(ncclGetUniqueId(&id)) != SWIM_OK) return SWIM_EDEVICE;
  std::memcpy(out, &id, sizeof(id));
  return SWIM_OK;
}

int32_t swim_create_shard(const swim_config* cfg, uint32_t capacity, uint32_t n_initial, uint64_t seed, int32_t rank,
                          int32_t world, const uint8_t* comm_id, swim_engine** out) {
  if (!cfg || (world > 1 && !comm_id)) return SWIM_EINVAL;
  // one rank without an id: the unsharded engine; one rank WITH an id: an RCCL engine of one rank,
  // which runs the whole exchange machinery (count collectives, the IPC mapping of its own region,
  // the row pulls, the quiet windows' allreduces) with nothing to exchange
  if (world <= 1 && !comm_id) return create_engine(cfg, capacity, n_initial, seed, 0, 1, false, nullptr, out);
  return create_engine(cfg, capacity, n_initial, seed, rank, world, true, comm_id, out);
}

int32_t swim_shard_info(const swim_engine* e, int32_t* rank, int32_t* world, uint32_t* lo, uint32_t* count) {
  if (!e) return SWIM_EINVAL;
  if (rank) *rank = e->rank;
  if (world) *world = e->world;
  if (lo) *lo = e->rccl ? e->sh[0].c.lo : 0;
  if (count) *count = e->rccl ? e->sh[0].c.nl : e->n;
  return SWIM_OK;
}

int32_t swim_exchange_info(const swim_engine* e, uint32_t* flags) {
  if (!e || !flags) return SWIM_EINVAL;
  uint32_t f = e->xflags;
  if (e->xchg) f |= SWIM_XCHG_ON;
  if (e->rccl) f |= SWIM_XCHG_RCCL;
  if (e->xchg && e->sh[0].xreg_uncached) f |= SWIM_XCHG_UNCACHED;
  *flags = f;
  return SWIM_OK;
}

int32_t swim_destroy(swim_engine* e) {
  delete e;
  return SWIM_OK;
}

static int32_t upload_member_seeds(swim_engine* e);
int32_t swim_step_ticks(swim_engine* e, uint32_t ticks) {
  if (!e) return SWIM_EINVAL;
  if (hipSetDevice(e->device) != hipSuccess) return SWIM_EDEVICE;
  bool fresh = false;  // the last work on the stream was a quiet window (status words written, drained)
  if (e->mseed_dirty)
    if (int32_t rc = upload_member_seeds(e)) return rc;
  for (uint32_t i = 0; i < ticks; ++i) {
    if (quiet_eligible(e) && e->T + 1 >= e->quiet_retry_at) {
      const uint32_t K = std::min(ticks - i, kQuietMax);
      uint32_t done = 0;
      if (int32_t rc = run_quiet(e, K, &done)) return rc;
      fresh = true;
      i += done;
      if (done == K) {
        e->quiet_backoff = 1;
        --i;  // (the loop's ++i)
        continue;
      }
      // the tick the window stopped at needs the per-tick chain; a window that advanced nothing means
      // the cluster is busy: the next try backs off
      e->quiet_backoff = done ? 1u : std::min(2 * e->quiet_backoff, kQuietBackoffMax);
      e->quiet_retry_at = e->T + 1 + e->quiet_backoff;
      if (i >= ticks) break;
    }
    if (int32_t rc = run_tick(e)) return rc;
    fresh = false;
    if (++e->since_drain >= e->drain_every) {
      int32_t r = sync_and_collect(e);
      if (r == SWIM_EDEVICE) return r;
    }
  }
  if (hip_status() != SWIM_OK) return SWIM_EDEVICE;
  int32_t rc = sync_and_collect(e, fresh);
  if (rc == SWIM_EDEVICE) return rc;
  if (e->rccl) {  // every rank reports a capacity error if any rank saw one
    uint32_t mine = e->err_seen ? 1u : 0u, any = 0;
    hipMemcpy(e->d_cnt, &mine, 4, hipMemcpyHostToDevice);
    if (nccl_ok(ncclAllReduce(e->d_cnt, e->d_cnt + 1, 1, ncclUint32, ncclMax, e->comm, e->stream)) != SWIM_OK)
      return SWIM_EDEVICE;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
    hipMemcpy(&any, e->d_cnt + 1, 4, hipMemcpyDeviceToHost);
    if (any) rc = SWIM_ECAPACITY;
  }
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
  mutated(e);  // (the precomputed quiet window no longer holds)
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
  for (Shard& sd : e->sh) {
    if (!s.empty() && hipMemcpy(sd.c.seeds, s.data(), 4 * s.size(), hipMemcpyHostToDevice) != hipSuccess)
      return SWIM_EDEVICE;
    if (hipMemcpy(sd.c.is_seed, e->is_seed_h.data(), e->n, hipMemcpyHostToDevice) != hipSuccess) return SWIM_EDEVICE;
    sd.c.n_seeds = (uint32_t)s.size();
  }
  return SWIM_OK;
}

int32_t swim_set_member_seeds(swim_engine* e, uint32_t m, const uint32_t* seeds, uint32_t n_seeds) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || m >= e->n) return SWIM_EINVAL;
  if (e->mseed_own_h.empty()) {
    e->mseed_own_h.assign(e->n, 0);
    e->mseeds_h.assign(e->n, {});
  }
  if (!seeds && n_seeds == 0xffffffffu) {  // back on the engine-wide list
    e->mseed_own_h[m] = 0;
    e->mseeds_h[m].clear();
    e->mseed_dirty = true;
    return SWIM_OK;
  }
  if (n_seeds && !seeds) return SWIM_EINVAL;
  std::vector<uint32_t> s;
  for (uint32_t i = 0; i < n_seeds; ++i) {
    if (seeds[i] >= e->n) return SWIM_EINVAL;
    if (std::find(s.begin(), s.end(), seeds[i]) == s.end()) s.push_back(seeds[i]);  // LinkedHashSet
  }
  e->mseeds_h[m] = std::move(s);
  e->mseed_own_h[m] = 1;
  e->mseed_dirty = true;
  return SWIM_OK;
}

// the per-member seed lists as CSR (own flags, offsets, members) on every shard (replicated)
static int32_t upload_member_seeds(swim_engine* e) {
  const uint32_t n = e->n;
  std::vector<uint32_t> off(n + 1, 0), all;
  for (uint32_t v = 0; v < n; ++v) {
    off[v] = (uint32_t)all.size();
    all.insert(all.end(), e->mseeds_h[v].begin(), e->mseeds_h[v].end());
  }
  off[n] = (uint32_t)all.size();
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  for (Shard& sd : e->sh) {
    uint8_t* own = const_cast<uint8_t*>(sd.c.mseed_own);
    uint32_t* o = const_cast<uint32_t*>(sd.c.mseed_off);
    uint32_t* l = const_cast<uint32_t*>(sd.c.mseed);
    if (!own) {
      if (!sd.alloc(&own, n) || !sd.alloc(&o, n + 1)) return SWIM_ENOMEM;
      sd.c.mseed_own = own;
      sd.c.mseed_off = o;
    }
    if (all.size() > sd.mseed_cap) {
      const size_t cap = std::max<size_t>(all.size(), 2 * sd.mseed_cap);
      uint32_t* fresh = nullptr;
      if (!sd.alloc(&fresh, cap)) return SWIM_ENOMEM;  // (the old list stays: the retry finds it)
      sd.release(l);
      l = fresh;
      sd.mseed_cap = cap;
      sd.c.mseed = l;
    }
    if (hipMemcpy(own, e->mseed_own_h.data(), n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(o, off.data(), 4ull * (n + 1), hipMemcpyHostToDevice) != hipSuccess ||
        (!all.empty() && hipMemcpy(l, all.data(), 4ull * all.size(), hipMemcpyHostToDevice) != hipSuccess))
      return SWIM_EDEVICE;
  }
  // (cleared only once every shard holds the new lists: a failure above leaves it set, and the next
  // swim_step uploads every shard again)
  e->mseed_dirty = false;
  return SWIM_OK;
}

int32_t swim_kill(swim_engine* e, uint32_t m) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || m >= e->n) return SWIM_EINVAL;
  e->pristine = false;
  uint8_t up = 0;
  if (read_up(e, m, &up) != SWIM_OK) return SWIM_EDEVICE;
  if (!up) return SWIM_ESTATE;
  if (set_replicated(e, offsetof(Ctx, up), m, 0, false) != SWIM_OK) return SWIM_EDEVICE;
  if (Shard* sd = e->owner_of(m)) {
    MemberDev md;
    if (read_member_dev(e, *sd, m, &md) != SWIM_OK) return SWIM_EDEVICE;
    md.leave_pending = 0;
    return write_member_dev(*sd, m, md);
  }
  return SWIM_OK;
}

int32_t swim_leave(swim_engine* e, uint32_t m, int32_t stop_after) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || m >= e->n) return SWIM_EINVAL;
  e->pristine = false;
  uint8_t up = 0;
  if (read_up(e, m, &up) != SWIM_OK) return SWIM_EDEVICE;
  if (!up) return SWIM_ESTATE;
  Shard* sd = e->owner_of(m);
  if (!sd) return SWIM_OK;  // RCCL: the owning rank runs it
  sd->c.T = e->T;
  k_leave<<<1, 64, 0, e->stream>>>(sd->c, m, stop_after);
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return hip_status();
}

int32_t swim_update_metadata(swim_engine* e, uint32_t m) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || m >= e->n) return SWIM_EINVAL;
  uint8_t up = 0;
  if (read_up(e, m, &up) != SWIM_OK) return SWIM_EDEVICE;
  if (!up) return SWIM_ESTATE;
  for (Shard& sd : e->sh) {
    if (!sd.c.meta_seen) {  // every store still holds version 0 of everything
      uint32_t* p = nullptr;
      if (!sd.alloc(&p, (size_t)std::max(sd.c.nl, 1u) * e->n)) return SWIM_ENOMEM;
      if (hipMemsetAsync(p, 0, 4ull * std::max(sd.c.nl, 1u) * e->n, e->stream) != hipSuccess) return SWIM_EDEVICE;
      sd.c.meta_seen = p;
    }
    sd.c.T = e->T;
    k_update_meta<<<1, 64, 0, e->stream>>>(sd.c, m, e->owner_of(m) == &sd ? 1 : 0);
  }
  return hip_status();
}

int32_t swim_set_namespaces(swim_engine* e, const uint16_t* ns_of_member, uint32_t n_ns, const uint8_t* related) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e) return SWIM_EINVAL;
  if (n_ns == 0 || !ns_of_member) {
    for (Shard& sd : e->sh) sd.c.n_ns = 0;
    return SWIM_OK;
  }
  if (!related || n_ns > 4096) return SWIM_EINVAL;
  for (uint32_t i = 0; i < e->n; ++i)
    if (ns_of_member[i] >= n_ns) return SWIM_EINVAL;
  std::vector<uint8_t> used(n_ns, 0);  // the converged start holds every initial member everywhere
  for (uint32_t a = 0; a < e->n; ++a)
    if (e->joined_h[a]) used[ns_of_member[a]] = 1;
  for (uint32_t x = 0; x < n_ns; ++x)
    for (uint32_t y = 0; y < n_ns; ++y)
      if (used[x] && used[y] && !related[(size_t)x * n_ns + y]) return SWIM_ESTATE;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  for (Shard& sd : e->sh) {
    uint16_t* ns = nullptr;
    uint8_t* rel = nullptr;
    if (!sd.alloc(&ns, e->n) || !sd.alloc(&rel, (size_t)n_ns * n_ns)) return SWIM_ENOMEM;
    if (hipMemcpy(ns, ns_of_member, 2ull * e->n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(rel, related, (size_t)n_ns * n_ns, hipMemcpyHostToDevice) != hipSuccess)
      return SWIM_EDEVICE;
    sd.c.ns = ns;
    sd.c.ns_rel = rel;
    sd.c.n_ns = n_ns;
  }
  return SWIM_OK;
}

int32_t swim_spread(swim_engine* e, uint32_t m, uint32_t payload) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || m >= e->n) return SWIM_EINVAL;
  uint8_t up = 0;
  if (read_up(e, m, &up) != SWIM_OK) return SWIM_EDEVICE;
  if (!up) return SWIM_ESTATE;
  Shard* sd = e->owner_of(m);
  if (!sd) return SWIM_OK;  // RCCL: the owning rank runs it
  sd->c.T = e->T;
  k_spread<<<1, 64, 0, e->stream>>>(sd->c, m, payload);
  return hip_status();
}

int32_t swim_ingest_sync(swim_engine* e, uint32_t v, const swim_record* records, uint32_t n, int32_t initial) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || v >= e->n || n > e->n || (n && !records)) return SWIM_EINVAL;
  e->pristine = false;
  for (uint32_t i = 0; i < n; ++i)
    if (records[i].member >= e->n || records[i].status >= SWIM_DEAD || records[i].inc < 0) return SWIM_EINVAL;
  uint8_t up = 0;
  if (read_up(e, v, &up) != SWIM_OK) return SWIM_EDEVICE;
  if (!up) return SWIM_ESTATE;
  Shard* sd = e->owner_of(v);
  if (!sd) return SWIM_OK;  // RCCL: the owning rank applies it
  swim_record* d = nullptr;
  if (hipMalloc((void**)&d, sizeof(swim_record) * std::max(n, 1u)) != hipSuccess) return SWIM_ENOMEM;
  int32_t rc = SWIM_OK;
  sd->c.T = e->T;
  sync_params(e, *sd);
  if (n && hipMemcpy(d, records, sizeof(swim_record) * n, hipMemcpyHostToDevice) != hipSuccess) rc = SWIM_EDEVICE;
  if (rc == SWIM_OK) {
    k_ingest_sync<<<1, 256, 0, e->stream>>>(sd->d_par, e->T, v, d, n, initial);
    if (hipStreamSynchronize(e->stream) != hipSuccess) rc = SWIM_EDEVICE;
    e->par_slot = 0;
  }
  hipFree(d);
  return rc == SWIM_OK ? hip_status() : rc;
}

int32_t swim_join(swim_engine* e, uint32_t m) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || m >= e->n) return SWIM_EINVAL;
  uint8_t up = 0;
  if (read_up(e, m, &up) != SWIM_OK) return SWIM_EDEVICE;
  if (e->joined_h[m] || up || e->join_pending_h[m]) return SWIM_ESTATE;
  if (Shard* sd = e->owner_of(m)) {
    MemberDev md;
    if (read_member_dev(e, *sd, m, &md) != SWIM_OK) return SWIM_EDEVICE;
    md.join_pending = 1;
    if (write_member_dev(*sd, m, md) != SWIM_OK) return SWIM_EDEVICE;
  }
  e->joined_h[m] = 1;
  e->joins.push_back(m);
  e->g_residue[(e->T + 1) % e->G] = 1;  // the joiner's gossip timer phase
  return SWIM_OK;
}

int32_t swim_join_at(swim_engine* e, uint32_t m, uint32_t addr_of) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || m >= e->n || addr_of >= e->n || addr_of == m) return SWIM_EINVAL;
  e->pristine = false;
  const uint32_t holder = e->route_of(addr_of);
  uint8_t up = 0;
  if (read_up(e, holder, &up) != SWIM_OK) return SWIM_EDEVICE;
  if (up || std::find(e->joins.begin(), e->joins.end(), holder) != e->joins.end()) return SWIM_ESTATE;
  for (auto& bd : e->binds)
    if (e->route_of(bd.second) == holder) return SWIM_ESTATE;  // the address is taken at the next tick
  if (int32_t rc = swim_join(e, m)) return rc;
  e->binds.push_back({m, addr_of});
  return SWIM_OK;
}

int32_t swim_set_default_loss(swim_engine* e, uint32_t m, int32_t pct) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || pct < 0 || pct > 100) return SWIM_EINVAL;
  if (m != 0xffffffffu && m >= e->n) return SWIM_EINVAL;
  const int32_t rc = set_replicated(e, offsetof(Ctx, default_loss), m, (uint8_t)pct, m == 0xffffffffu);
  if (rc != SWIM_OK) return rc;
  if (m == 0xffffffffu) {
    std::fill(e->loss_h.begin(), e->loss_h.end(), (uint8_t)pct);
    e->loss_nz = pct ? e->n : 0;
  } else {
    e->loss_nz += (pct != 0 ? 1 : 0) - (e->loss_h[m] != 0 ? 1 : 0);
    e->loss_h[m] = (uint8_t)pct;
  }
  return SWIM_OK;
}

int32_t swim_set_link_loss(swim_engine* e, uint32_t src, uint32_t dst, int32_t pct) {
  mutated(e);  // (the precomputed quiet window no longer holds)
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

// ---- message delay (swim_delay.h): one threshold table per distinct meanDelay, on every shard.
// The tables live in one device array that grows by doubling (the previous one is freed after the
// stream drained), and only the new table is written.  A mean above SWIM_DELAY_MEAN_MAX_TICKS ticks
// is refused: beyond it the SWIM_DELAY_TICKS_MAX cap would truncate draws with non-negligible
// probability (swim_delay_mean_ok, shared with the oracle).
// whether delay_table would accept mean_ms: checked before any state changes (a refused mean must
// leave the engine exactly as it was, as the oracle's setter does)
static bool delay_mean_acceptable(const swim_engine* e, int32_t mean_ms) {
  if (!swim_delay_mean_ok(mean_ms, e->tick_ms)) return false;
  for (int32_t m : e->delay_means)
    if (m == mean_ms) return true;
  return e->delay_means.size() < 4096;
}
static int32_t delay_table(swim_engine* e, int32_t mean_ms, int32_t* idx) {
  for (size_t i = 0; i < e->delay_means.size(); ++i)
    if (e->delay_means[i] == mean_ms) { *idx = (int32_t)i; return SWIM_OK; }
  if (!delay_mean_acceptable(e, mean_ms)) return SWIM_EINVAL;
  std::vector<uint64_t> th(SWIM_DELAY_TICKS_MAX);
  swim_delay_thresholds(mean_ms, e->tick_ms, th.data());
  const size_t nt = e->delay_means.size() + 1;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  for (Shard& sd : e->sh) {
    if (!sd.grow(&sd.delay_buf, &sd.delay_cap, nt * SWIM_DELAY_TICKS_MAX, /*keep=*/true)) return SWIM_ENOMEM;
    sd.c.delay_th = sd.delay_buf;
    if (hipMemcpy(sd.delay_buf + (nt - 1) * SWIM_DELAY_TICKS_MAX, th.data(), 8 * th.size(), hipMemcpyHostToDevice) !=
        hipSuccess)
      return SWIM_EDEVICE;
  }
  e->delay_means.push_back(mean_ms);
  *idx = (int32_t)(nt - 1);
  return SWIM_OK;
}
// the delay rings and the per-tick release are set up on every shard the first time a delay is
// configured.  A delayed message waits in its SENDER's shard and joins the exchange of its arrival
// tick (GOSSIP_REQs: k_dq_release; SYNC / SYNC_ACK: k_sync_delay), so sharded engines need nothing more.
static int32_t enable_delay(swim_engine* e) {
  if (e->n > (1u << 20)) return SWIM_EINVAL;  // (a released GOSSIP_REQ carries its age above bit 20 of `from`)
  for (Shard& sd : e->sh) {
    if (sd.c.delay_on) continue;
    const uint32_t bcap = e->cfg.delay_capacity ? e->cfg.delay_capacity : 1024;
    GMsgFull* dq = nullptr;
    if (!sd.alloc(&dq, (size_t)DQ_BUCKETS * bcap)) return SWIM_ENOMEM;
    sd.b.dq = dq;
    sd.b.dq_bcap = bcap;
    // delayed SYNCs / SYNC_ACKs: a bucket holds a few ticks' worth of SYNCs (N / S per tick, and as
    // many acks); every message in flight parks its content row (at most 1 GiB of rows)
    const uint32_t per_tick = (e->n + sd.c.S - 1) / std::max(sd.c.S, 1u);
    const uint32_t sbcap = 64 + 8 * per_tick;
    const uint32_t pcap = (uint32_t)std::min<uint64_t>(4ull * sbcap, std::max<uint64_t>(64, (1ull << 28) / e->n));
    Bufs& b = sd.b;
    if (!sd.alloc(&b.sdq, (size_t)DQ_BUCKETS * sbcap) || !sd.alloc(&b.sdq_cnt, DQ_BUCKETS) ||
        !sd.alloc(&b.park, (size_t)pcap * e->n) || !sd.alloc(&b.park_avail, pcap) || !sd.alloc(&b.park_freed, pcap) ||
        !sd.alloc(&b.park_jobs, pcap) || !sd.alloc(&b.park_ctl, 1))
      return SWIM_ENOMEM;
    if (hipMemset(b.sdq_cnt, 0, 4ull * DQ_BUCKETS) != hipSuccess || hipMemset(b.park_ctl, 0, sizeof(SpillCtl)) != hipSuccess)
      return SWIM_EDEVICE;
    b.sdq_bcap = sbcap;
    b.park_cap = pcap;
    // delayed metadata round trips: the base capacity of a cluster that is not joining; a join
    // burst grows it before its tick (grow_for_joins)
    const uint32_t fcap = std::max<uint32_t>(4096, 2 * e->n);
    const size_t nl2 = 2ull * std::max(sd.c.nl, 1u);
    if (!sd.alloc(&sd.c.fq, 2ull * fcap) || !sd.alloc(&sd.c.fq_head, nl2) || !sd.alloc(&sd.c.fq_tail, nl2) ||
        !sd.alloc(&sd.c.fq_cnt, 2))
      return SWIM_ENOMEM;
    if (hipMemset(sd.c.fq_head, 0xff, 4 * nl2) != hipSuccess || hipMemset(sd.c.fq_cnt, 0, 8) != hipSuccess)
      return SWIM_EDEVICE;
    sd.c.fq_cap = fcap;
    sd.c.delay_on = 1;
  }
  return SWIM_OK;
}

int32_t swim_set_default_delay(swim_engine* e, uint32_t m, int32_t mean_ms) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || mean_ms < 0 || (m != 0xffffffffu && m >= e->n)) return SWIM_EINVAL;
  int32_t idx = -1;
  if (mean_ms > 0) {
    if (!delay_mean_acceptable(e, mean_ms)) return SWIM_EINVAL;
    if (int32_t rc = enable_delay(e)) return rc;
    if (int32_t rc = delay_table(e, mean_ms, &idx)) return rc;
  }
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  for (Shard& sd : e->sh) {
    const int16_t v = (int16_t)idx;
    hipError_t r = m == 0xffffffffu ? hipMemsetD16(reinterpret_cast<hipDeviceptr_t>(sd.c.default_delay), (uint16_t)v, e->n)
                                    : hipMemcpy(sd.c.default_delay + m, &v, 2, hipMemcpyHostToDevice);
    if (r != hipSuccess) return SWIM_EDEVICE;
  }
  return SWIM_OK;
}

int32_t swim_set_link_delay(swim_engine* e, uint32_t src, uint32_t dst, int32_t mean_ms) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || src >= e->n || dst >= e->n) return SWIM_EINVAL;
  int32_t idx = mean_ms < 0 ? -1 : -2;
  if (mean_ms > 0) {
    if (!delay_mean_acceptable(e, mean_ms)) return SWIM_EINVAL;
    if (int32_t rc = enable_delay(e)) return rc;
    if (int32_t rc = delay_table(e, mean_ms, &idx)) return rc;
  }
  if (idx == -1) {
    LinkDev* L = find_link_h(e, src, dst, false);
    if (L) L->out_delay = -1;
  } else {
    find_link_h(e, src, dst, true)->out_delay = idx;
  }
  prune_links(e);
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  return upload_links(e);
}

int32_t swim_set_link_inbound(swim_engine* e, uint32_t dst, uint32_t src, int32_t pass) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e || src >= e->n || dst >= e->n) return SWIM_EINVAL;
  e->pristine = false;
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
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e) return SWIM_EINVAL;
  e->pristine = false;
  if (m != 0xffffffffu && m >= e->n) return SWIM_EINVAL;
  return set_replicated(e, offsetof(Ctx, default_inbound), m, pass ? 1 : 0, m == 0xffffffffu);
}

int32_t swim_set_partition(swim_engine* e, const uint16_t* g) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  for (Shard& sd : e->sh) {
    if (!g) { sd.c.partition = 0; continue; }
    if (hipMemcpy(sd.c.group, g, 2 * (size_t)e->n, hipMemcpyHostToDevice) != hipSuccess) return SWIM_EDEVICE;
    sd.c.partition = 1;
  }
  return SWIM_OK;
}

int32_t swim_read_view(swim_engine* e, uint32_t v, uint64_t* out) {
  if (!e || v >= e->n || !out) return SWIM_EINVAL;
  Shard* sd = e->owner_of(v);
  if (!sd) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  // compose the swim.h packed cells from the split record / aux words (swim_device.h)
  std::vector<uint32_t> r(e->n), a(e->n);
  const size_t off = (size_t)(v - sd->c.lo) * e->n;
  if (hipMemcpy(r.data(), sd->c.recs + off, 4 * (size_t)e->n, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(a.data(), sd->c.aux + off, 4 * (size_t)e->n, hipMemcpyDeviceToHost) != hipSuccess)
    return SWIM_EDEVICE;
  for (uint32_t x = 0; x < e->n; ++x)
    out[x] = (uint64_t)(r[x] & REC_INC_MASK) | ((uint64_t)((r[x] >> 29) & 3u) << 32) | ((uint64_t)(r[x] >> 31) << 34) |
             ((uint64_t)(a[x] & 0xfu) << 35) | ((uint64_t)(a[x] >> 4) << 39);
  return SWIM_OK;
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
  for (int r = 0; r < 7; ++r) out->gossips_by_reason[r] = st[ST_ORIG0 + r];
  return SWIM_OK;
}

int32_t swim_read_member(swim_engine* e, uint32_t v, swim_member_state* o) {
  if (!e || v >= e->n || !o) return SWIM_EINVAL;
  Shard* sd = e->owner_of(v);
  if (!sd) return SWIM_EINVAL;
  MemberDev m;
  GossipSched gs;
  if (read_member_dev(e, *sd, v, &m) != SWIM_OK || read_gsched(*sd, v, &gs) != SWIM_OK) return SWIM_EDEVICE;
  uint8_t up = 0;
  if (read_up(e, v, &up) != SWIM_OK) return SWIM_EDEVICE;
  std::memset(o, 0, sizeof(*o));
  o->up = up;
  o->joined = m.joined;
  o->leave_pending = m.leave_pending;
  o->join_pending = m.join_pending;
  o->remote_idx = m.remote_idx;
  o->fd_period = m.fd_period;
  o->ping_cursor = m.ping_cursor;
  o->ping_len = m.ping_len;
  o->remote_len = m.remote_len;
  o->gossip_len = gs.len;
  o->gossip_period = gs.period;
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
  uint32_t pn = 0;
  if (hipMemcpy(&pn, sd->c.pa_n + (v - sd->c.lo), 4, hipMemcpyDeviceToHost) != hipSuccess) return SWIM_EDEVICE;
  o->pending_acks = pn;
  return SWIM_OK;
}

static int32_t read_list(swim_engine* e, Shard& sd, uint32_t v, const uint32_t* base, uint32_t len, uint32_t* out,
                         uint32_t cap, uint32_t* lenp) {
  if (lenp) *lenp = len;
  if (out && cap && len) {
    uint32_t k = std::min(cap, len);
    if (hipMemcpy(out, base + (size_t)(v - sd.c.lo) * e->n, 4 * (size_t)k, hipMemcpyDeviceToHost) != hipSuccess)
      return SWIM_EDEVICE;
  }
  return SWIM_OK;
}

int32_t swim_read_ping_list(swim_engine* e, uint32_t v, uint32_t* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  Shard* sd = e->owner_of(v);
  if (!sd) return SWIM_EINVAL;
  MemberDev m;
  if (read_member_dev(e, *sd, v, &m) != SWIM_OK) return SWIM_EDEVICE;
  return read_list(e, *sd, v, sd->c.ping, m.ping_len, out, cap, len);
}

int32_t swim_read_remote_list(swim_engine* e, uint32_t v, uint32_t* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  Shard* sd = e->owner_of(v);
  if (!sd) return SWIM_EINVAL;
  MemberDev m;
  if (read_member_dev(e, *sd, v, &m) != SWIM_OK) return SWIM_EDEVICE;
  return read_list(e, *sd, v, sd->c.remote, m.remote_len, out, cap, len);
}

int32_t swim_read_gossips(swim_engine* e, uint32_t v, swim_gossip* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  Shard* sd = e->owner_of(v);
  if (!sd) return SWIM_EINVAL;
  GossipSched gs;
  if (hipStreamSynchronize(e->stream) != hipSuccess || read_gsched(*sd, v, &gs) != SWIM_OK) return SWIM_EDEVICE;
  if (len) *len = gs.len;
  uint32_t k = std::min(cap, gs.len);
  if (!out || !k) return SWIM_OK;
  std::vector<GossipHot> gh(k);
  std::vector<GossipCold> gc(k);
  const size_t o = (size_t)(v - sd->c.lo) * sd->c.gcap;
  // the slab is a ring from gs.base (swim_device.h SlabRef): at most two segments
  const uint32_t start = gs.base & (sd->c.gcap - 1), first = std::min(k, sd->c.gcap - start);
  if (hipMemcpy(gh.data(), sd->c.slab_hot + o + start, sizeof(GossipHot) * first, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(gc.data(), sd->c.slab_cold + o + start, sizeof(GossipCold) * first, hipMemcpyDeviceToHost) != hipSuccess ||
      (k > first &&
       (hipMemcpy(gh.data() + first, sd->c.slab_hot + o, sizeof(GossipHot) * (k - first), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(gc.data() + first, sd->c.slab_cold + o, sizeof(GossipCold) * (k - first), hipMemcpyDeviceToHost) != hipSuccess)))
    return SWIM_EDEVICE;
  std::vector<InfOver> io;  // the member's infected overflows, read when a state has one
  for (uint32_t i = 0; i < k; ++i) {  // (the SlabRef layout, swim_device.h)
    out[i].gossiper = gh[i].gossiper;
    out[i].subject = gc[i].subject;
    out[i].seq = gh[i].seq;
    out[i].inc = gc[i].inc;
    out[i].status = (gh[i].per_st >> PER_BITS) & 7u;
    out[i].infection_period = gh[i].per_st & PER_MASK;
    out[i].infected[0] = gh[i].inf0;
    out[i].infected[1] = NONE;
    if (gh[i].per_st >> 31) {
      const uint32_t cap = sd->c.inf_mask + 1;
      if (io.empty()) {
        io.resize(cap);
        if (hipMemcpy(io.data(), sd->c.inf_over + (size_t)(v - sd->c.lo) * cap, sizeof(InfOver) * cap,
                      hipMemcpyDeviceToHost) != hipSuccess)
          return SWIM_EDEVICE;
      }
      for (uint32_t j = 0; j < cap; ++j)
        if (io[j].gossiper == gh[i].gossiper && io[j].seq == gh[i].seq) { out[i].infected[1] = io[j].inf[0]; break; }
    }
  }
  return SWIM_OK;
}

int32_t swim_read_collector(swim_engine* e, uint32_t v, uint32_t gossiper, swim_interval* out, uint32_t cap, uint32_t* len) {
  if (!e || v >= e->n) return SWIM_EINVAL;
  Shard* sd = e->owner_of(v);
  if (!sd) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  std::vector<CollEnt> tab(sd->c.hcap);
  if (hipMemcpy(tab.data(), sd->c.coll + (size_t)(v - sd->c.lo) * sd->c.hcap, sizeof(CollEnt) * sd->c.hcap,
                hipMemcpyDeviceToHost) != hipSuccess)
    return SWIM_EDEVICE;
  if (len) *len = 0;
  for (const CollEnt& d : tab) {
    if (d.key != gossiper + 1) continue;
    const uint32_t n = d.meta & 7u;
    std::vector<uint32_t> blk;
    if (n == COLL_SPILLED) {
      const int t = (int)((d.meta >> 4) & 3u);
      blk.resize(tier_words(t));
      if (hipMemcpy(blk.data(), sd->c.spill[t] + (size_t)(d.meta >> 8) * tier_words(t), 4 * blk.size(),
                    hipMemcpyDeviceToHost) != hipSuccess)
        return SWIM_EDEVICE;
    }
    const uint32_t cnt = n == COLL_SPILLED ? blk[0] : n;
    if (len) *len = cnt;
    for (uint32_t i = 0; i < cnt && i < cap && out; ++i) {
      out[i].lo = n == COLL_SPILLED ? blk[4 + 2 * i] : d.lo;
      out[i].hi = n == COLL_SPILLED ? blk[5 + 2 * i] : d.hi;
    }
    break;
  }
  return SWIM_OK;
}

int32_t swim_set_quiet_path(swim_engine* e, int32_t enable) {
  mutated(e);  // (the precomputed quiet window no longer holds)
  if (!e) return SWIM_EINVAL;
  e->quiet_on = enable != 0;
  e->quiet_retry_at = 0;
  e->quiet_backoff = 1;
  return SWIM_OK;
}

int32_t swim_get_quiet_stats(const swim_engine* e, swim_quiet_stats* out) {
  if (!e || !out) return SWIM_EINVAL;
  *out = e->qst;
  return SWIM_OK;
}

int32_t swim_profile_quiet(swim_engine* e, swim_kernel_profile* out) {
  if (!e || !out) return SWIM_EINVAL;
  qev_flush(e);
  std::memset(out, 0, sizeof(*out));
  out->launches = e->qprof_windows;
  out->total_ms = e->qprof_ms;
  out->messages = e->qprof_ticks;
  out->records = e->qprof_mp;
  out->alg_bytes = e->qprof_bytes;
  return SWIM_OK;
}

int32_t swim_profile_enable(swim_engine* e, int32_t enable) {
  if (!e) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  for (hipEvent_t& ev : e->qev)
    if (!ev && hipEventCreate(&ev) != hipSuccess) return SWIM_EDEVICE;
  e->qev_n = 0;
  e->qprof_ms = 0.0;
  e->qprof_windows = e->qprof_ticks = e->qprof_mp = e->qprof_bytes = 0;
  for (Shard& sd : e->sh) {
    for (KProf* k : {&sd.prof_cls, &sd.prof_emit, &sd.prof_dlv}) {
      if (k->ev.empty()) {
        k->ev.resize(4 * kDrainEvery + 4);
        for (auto& ev : k->ev)
          if (hipEventCreate(&ev) != hipSuccess) return SWIM_EDEVICE;
        if (!sd.alloc(&k->slots, 3 * k->ev.size())) return SWIM_ENOMEM;
      }
      k->reset();
    }
  }
  e->prof = enable != 0;
  return SWIM_OK;
}

int32_t swim_profile_merge(swim_engine* e, swim_kernel_profile* out) {
  if (!e || !out) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  std::memset(out, 0, sizeof(*out));
  uint64_t units = 0;
  for (Shard& sd : e->sh) {
    sd.prof_cls.flush();
    out->launches += sd.prof_cls.launches;
    out->total_ms += sd.prof_cls.ms;
    out->messages += sd.prof_cls.a;
    out->records += sd.prof_cls.b;
    units += sd.prof_cls.c;
  }
  const uint64_t skipped = units > out->messages ? units - out->messages : 0;
  // per streamed unit the record words of both rows over its 1,024 subjects; per unit the block
  // witness skipped, its two block counts; per complex record its pool entry
  out->alg_bytes = out->messages * 8ull * SYNC_CHUNK + skipped * 8ull + out->records * 4ull;
  return SWIM_OK;
}

int32_t swim_profile_fanout(swim_engine* e, swim_kernel_profile* out) {
  if (!e || !out) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  std::memset(out, 0, sizeof(*out));
  for (Shard& sd : e->sh) {
    sd.prof_emit.flush();
    out->launches += sd.prof_emit.launches;
    out->total_ms += sd.prof_emit.ms;
    out->messages += sd.prof_emit.a;
    out->records += sd.prof_emit.b;
    out->examined += sd.prof_emit.c;
  }
  // SURVEY.md §8(d) fanout: 24 B per emitted GOSSIP_REQ + 32 B per (gossip, sender round) read
  out->alg_bytes = out->messages * 24ull + out->records * 32ull;
  return SWIM_OK;
}

int32_t swim_profile_deliver(swim_engine* e, swim_kernel_profile* out) {
  if (!e || !out) return SWIM_EINVAL;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return SWIM_EDEVICE;
  std::memset(out, 0, sizeof(*out));
  uint64_t fresh = 0;
  for (Shard& sd : e->sh) {
    sd.prof_dlv.flush();
    out->launches += sd.prof_dlv.launches;
    out->total_ms += sd.prof_dlv.ms;
    out->messages += sd.prof_dlv.a;
    fresh += sd.prof_dlv.b;
    out->records += sd.prof_dlv.c;
  }
  // SURVEY.md §8(d) merge: 24 B per delivered GOSSIP_REQ read, + 8 B dedupe RMW + 16 B view RMW per
  // message that runs onGossipReq's collector check (those emit flagged as provable duplicates do not)
  out->alg_bytes = out->messages * 24ull + fresh * 24ull;
  return SWIM_OK;
}

// profiling builds (-DSWIM_PHASE_PROF): the per-phase wall-time sums of the instrumented kernels
// (swim_phases.h g_dbg); reset = 1 zeroes them after the read.  Zeros in the product build.
int32_t swim_debug_counters(uint64_t* out, uint32_t n, int32_t reset) {
  if (!out || n > 64) return SWIM_EINVAL;
  unsigned long long h[64] = {};
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dbg), sizeof h) != hipSuccess)
    return SWIM_EDEVICE;
  for (uint32_t i = 0; i < n; ++i) out[i] = h[i];
  if (reset) {
    unsigned long long z[64] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof z) != hipSuccess) return SWIM_EDEVICE;
  }
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
  CollEnt* de = nullptr;
  uint32_t* dsp = nullptr;  // one block per tier + the tier bookkeeping
  uint32_t* derr = nullptr;
  // frees are recycled only at a tick end, so every spill of the run gets a fresh block
  uint32_t kcap[NTIER];
  size_t words = 0;
  for (int t = 0; t < NTIER; ++t) {
    kcap[t] = t < 2 ? n : std::min<uint32_t>(n, 8);
    words += (size_t)kcap[t] * (tier_words(t) + 2);
  }
  if (hipMalloc((void**)&dk, n) != hipSuccess || hipMalloc((void**)&dv, 8 * (size_t)n) != hipSuccess ||
      hipMalloc((void**)&dr, 8 * (size_t)n) != hipSuccess || hipMalloc((void**)&de, sizeof(CollEnt)) != hipSuccess ||
      hipMalloc((void**)&dsp, 4 * words) != hipSuccess ||
      hipMalloc((void**)&derr, 4 + sizeof(SpillCtl) * NTIER) != hipSuccess)
    return SWIM_EDEVICE;
  hipMemcpy(dk, kinds, n, hipMemcpyHostToDevice);
  hipMemcpy(dv, values, 8 * (size_t)n, hipMemcpyHostToDevice);
  hipMemset(derr, 0, 4 + sizeof(SpillCtl) * NTIER);
  Ctx c{};
  c.err = derr;
  c.spill_ctl = reinterpret_cast<SpillCtl*>(derr + 1);
  c.seg_threshold = INT32_MAX;
  uint32_t* p = dsp;
  for (int t = 0; t < NTIER; ++t) {
    c.spill[t] = p; p += (size_t)kcap[t] * tier_words(t);
    c.spill_avail[t] = p; p += kcap[t];
    c.spill_freed[t] = p; p += kcap[t];
    c.spill_cap[t] = kcap[t];
  }
  k_kat_collector<<<1, 64>>>(c, dk, dv, n, dr, de);
  hipError_t r = hipMemcpy(results, dr, 8 * (size_t)n, hipMemcpyDeviceToHost);
  uint32_t err = 0;
  hipMemcpy(&err, derr, 4, hipMemcpyDeviceToHost);
  hipFree(dk); hipFree(dv); hipFree(dr); hipFree(de); hipFree(dsp); hipFree(derr);
  if (r != hipSuccess) return SWIM_EDEVICE;
  return err ? SWIM_ECAPACITY : hip_status();
}

}  // extern "C"
