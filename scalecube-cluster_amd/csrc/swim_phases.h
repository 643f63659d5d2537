// swim_kernels.h — the HIP kernels of one lockstep tick.
//
// Phase A  k_fd (per 256-viewer block)                suspicion timeouts
// Phase B  k_fd                                       list compaction after REMOVED, then ping /
//                                                     ping-req / ack resolution + FD events
// Phase C  round start (+ segmentation) in k_fd, k_gossip_emit (+ k_recv_msgs), k_gossip_deliver
// Phase D  SYNC collection (in k_fd / k_gossip_deliver), k_sync_prep, k_sync_classify, k_sync_apply (swim_sync.h; SYNC and SYNC_ACK)
// lists    (k_gossip_deliver, k_sync_apply)           deferred pingMembers inserts of ADDED events
// tick end k_end_tick
//
// Every kernel reads its work size from device memory (grid-stride over device counters), so the
// host never synchronises inside a tick.
#pragma once
#include "swim_device.h"

namespace swimdev {

// Phase timing for profiling builds only (-DSWIM_PHASE_PROF, tools/phase_prof.sh): per-wave wall
// time (s_memrealtime, 100 MHz) of the delivery kernel's parts, summed into g_dbg; read with
// swim_debug_counters.  The product build compiles none of it.
__device__ unsigned long long g_dbg[64];
#ifdef SWIM_PHASE_PROF
#define PPROF_T0(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#define PPROF_ADD(slot, t0)                                                                          \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_dbg[slot], __builtin_amdgcn_s_memrealtime() - (t0)); \
  } while (0)
#define PPROF_CNT(slot, val)                                     \
  do {                                                           \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_dbg[slot], (val)); \
  } while (0)
// wave time of a section that runs with some lanes inactive: added by the wave's first active lane
#define PPROF_WADD(slot, t0)                                                                          \
  do {                                                                                               \
    if ((threadIdx.x & 63) == (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1)                 \
      atomicAdd(&g_dbg[slot], __builtin_amdgcn_s_memrealtime() - (t0));                              \
  } while (0)
// wave-local accumulation (added to g_dbg once, with PPROF_CNT): no atomic per loop iteration
#define PPROF_ACC(var, t0) var += __builtin_amdgcn_s_memrealtime() - (t0)
#else
#define PPROF_T0(v)
#define PPROF_ADD(slot, t0)
#define PPROF_CNT(slot, val)
#define PPROF_WADD(slot, t0)
#define PPROF_ACC(var, t0)
#endif

// per-tick scratch counters, zeroed by one hipMemsetAsync at the start of every tick
struct Counters {
  uint32_t msg_total, pg_cursor, park_jobs;  // messages materialised this round; inbox pages taken; SYNC rows to park
  uint32_t req_total, req_recv_cnt, req_pg;  // SYNC items, receivers, inbox pages taken
  uint32_t ack_total, ack_recv_cnt, ack_pg;  // the same for SYNC_ACKs
  uint32_t ins_total, pad1;   // overflow list-insert ops of the gossip phase
  uint32_t ins_total2, pad2;  // overflow list-insert ops of the SYNC phase
  uint32_t pool_cursor;  // complex-record pool of the SYNC classify kernel
  uint32_t sender_cnt;   // senders of this tick's gossip round with live gossips
  uint32_t big_cnt;      // receivers whose inbox takes the wave-parallel delivery path
  uint32_t pad;
};

// per-tick message counts by destination shard (sharded engines), zeroed by k_end_tick
constexpr int MAXW = 16;
struct Xc {
  uint32_t msg[MAXW], req[MAXW], ack[MAXW];
  uint32_t stop;
  uint32_t pad[3];
};

// Where this shard reads what the other shards produced for it.  Device pointers: a
// local group's peers are the other shards in this process; with RCCL they are the peers' exchange
// buffers mapped over xGMI (hipIpcOpenMemHandle), read with system-scope loads after the exchange's
// count collective, which no rank leaves before every rank's producers have finished.
struct Peers {
  const GMsgFull* msgs[MAXW];        // peer p's tx_msgs ([world][tx_msg_cap])
  const SyncReq* hdr[2][MAXW];       // peer p's tx_reqs / tx_acks ([world][tx_req_cap])
  const uint32_t* stops[MAXW];       // peer p's tx_stops
  const uint32_t* rows[2][MAXW];     // peer p's packed SYNC / SYNC_ACK content rows ([row_cap][n])
  const uint32_t* rows_in[2][MAXW];  // where content rows from p are read: p's rows (local group) or
                                     // this shard's pulled copy (RCCL)
  uint32_t* rx_rows[2];              // RCCL: the pulled copies, [world][row_cap][n]
  const Xc* x[MAXW];                 // local group: peer counters (RCCL: the counts arrive in rx_cnt)
  // the cross-shard receipt filter (local group: Bufs.rfilter; over RCCL these stay null): peer p's
  // receipt slots and bitmaps, its receivers' collector clear ticks, its bitmap words per slot
  const GSlot* gslot[MAXW];
  const uint32_t* gbits[MAXW];
  const uint32_t* clr_tick[MAXW];
};
// rx_cnt[kind][p]: what peer p produced for this shard this tick (kind 0 GOSSIP_REQs, 1 SYNCs,
// 2 SYNC_ACKs) and, kind 3, its completed graceful leaves (broadcast)
enum : uint32_t { XK_MSG = 0, XK_REQ = 1, XK_ACK = 2, XK_STOP = 3 };

constexpr uint32_t DQ_BUCKETS = 2048, DQ_MASK = DQ_BUCKETS - 1;  // delay ring (> SWIM_DELAY_TICKS_MAX)
static_assert(DQ_BUCKETS > SWIM_DELAY_TICKS_MAX, "a delayed message must not land in the current bucket");

struct Bufs {
  Counters* k;
  // cross-shard exchange; an unsharded engine (world == 1) never touches these
  Xc* x;
  GMsgFull* tx_msgs;  // [world][tx_msg_cap] GOSSIP_REQs for receivers owned by another shard
  uint32_t tx_msg_cap;
  SyncReq* tx_reqs;   // [world][tx_req_cap] SYNCs whose receiver is owned by another shard
  SyncReq* tx_acks;   // [world][tx_req_cap] SYNC_ACKs whose receiver is owned by another shard
  uint32_t tx_req_cap;
  uint32_t* tx_stops; // members whose graceful leave completed this tick (broadcast)
  uint32_t tx_stop_cap;
  uint32_t* tx_rows[2];  // [row_cap][n] content rows of the outgoing SYNCs / SYNC_ACKs (k_pack_rows)
  uint32_t row_cap;
  const Peers* peers;
  uint32_t rfilter;      // emit checks receivers on other shards against their receipt bits (Peers.gslot...)
  uint32_t* rx_cnt;      // [4][MAXW] (XK_*)
  uint32_t* rx_stops;    // [world * tx_stop_cap] other shards' completed leaves, applied by k_end_tick
  uint32_t* rx_stop_n;   // how many (zeroed by k_fd, set by k_recv_msgs)
  // paged gossip inboxes (inbox_page): message k of receiver i's round is pg_msgs[pg_tab[i][k / 64]][k % 64]
  GMsgFull* pg_msgs;   // [pg_cap][64]
  uint32_t* pg_perm;   // [pg_cap][64] big inboxes: canonical rank -> inbox position, same paging
  uint32_t* pg_tab;    // [nl][pg_max] page of each 64-message stretch of the inbox, NONE = none yet
  uint32_t pg_cap, pg_max;
  uint32_t msg_cap;
  uint32_t* msg_cnt;   // per receiver
  uint32_t* big_list;  // local indices of receivers with big inboxes (the writer that crosses wave_min)
  uint32_t* big_tick;  // per receiver: tick whose inbox took the wave-parallel path
  uint32_t wave_min;   // inboxes above this many messages take it (<= DLV_SORT)
  uint32_t coop_min;   // big inboxes of at least this many messages are delivered by the whole wave
  // GOSSIP_REQs delayed by the network emulator (swim_delay.h): bucket (arrival tick & DQ_MASK) holds
  // up to dq_bcap messages, .pad = the sending tick; released into the inboxes by k_dq_release
  GMsgFull* dq;        // [DQ_BUCKETS][dq_bcap]
  uint32_t* dq_cnt;    // [DQ_BUCKETS]
  uint32_t dq_bcap;
  // SYNCs / SYNC_ACKs delayed by the network emulator: bucket (arrival tick & DQ_MASK) holds up to
  // sdq_bcap messages (RQ_PARKED: .snap = the park slot holding the content as it was prepared, .pad
  // = the sending tick).  k_sync_delay copies this tick's delayed SYNC contents into their slots and
  // moves the arrivals into the inboxes; a SYNC_ACK's content is parked by its acker's workgroup.
  SyncReq* sdq;         // [DQ_BUCKETS][sdq_bcap]
  uint32_t* sdq_cnt;    // [DQ_BUCKETS]
  uint32_t sdq_bcap;
  uint32_t* park;       // [park_cap][n] content rows of the messages in flight
  uint32_t park_cap;
  uint32_t* park_avail; // [park_cap] reusable slots (refilled from park_freed by k_end_tick)
  uint32_t* park_freed; // [park_cap] slots whose message arrived this tick
  uint2* park_jobs;     // [park_cap] (slot, sender): SYNC content rows to copy this tick
  SpillCtl* park_ctl;   // (bump, avail, freed) of the slots
  // SYNC / SYNC_ACK sub-phases (swim_sync.h): items in enqueue order; a receiver's inbox is paged
  // like the gossip inboxes: its k-th message is item pool[tab[r][k / 64]][k % 64]
  SyncReq* reqs;
  uint32_t req_cap;
  uint32_t* req_cnt;    // per receiver
  uint32_t* req_recv;   // receivers, in order of their first message
  uint32_t* rq_inl;     // [nl][SY_INLINE] the first messages of each inbox (no page needed)
  uint32_t* rq_tab;     // [nl][sy_max] pages of the rest: message SY_INLINE + j is page j / 64, slot j % 64
  uint32_t* rq_pool;    // [sy_pool_cap][64]
  SyncReq* acks;
  uint32_t* ack_cnt;
  uint32_t* ack_recv;
  uint32_t* ack_inl;
  uint32_t* ack_tab;
  uint32_t* ack_pool;
  uint32_t sy_max, sy_pool_cap;
  // content snapshots (a row that is both read as a message's content and merged into in one
  // sub-phase): SYNC content claimed during collection (sflag), SYNC_ACK content copied by the
  // acker's own k_sync_apply workgroup; slots released by k_end_tick
  uint32_t* snap;       // [snap_cap][n] record rows
  uint32_t snap_cap;
  uint32_t* snap_idx;   // per member: SYNC-content slot or NONE
  uint32_t* ack_snap;   // per member: SYNC_ACK-content slot or NONE (the same slot as snap_idx)
  uint32_t* snap_ready; // per member: tick << 2 | 1 (2): the slot holds its SYNC (SYNC_ACK) content
  uint32_t* snap_list;  // [2][snap_cap] members holding slots, by tick parity
  uint32_t* snap_cnt;   // [2] slots taken, by tick parity
  uint32_t* sflag;      // per member: tick << SF_BITS | SF_* bits of this tick
  uint64_t* pend;       // per sync-apply workgroup: pending ALIVE admissions
  uint2* item_chunk;    // per (SYNC item, chunk): (pool base, complex count)
  uint32_t* item_total; // per SYNC item: complex count over all chunks
  uint2* ack_chunk;     // the same for SYNC_ACK items (classified by k_ack_classify when sharded)
  uint32_t* ack_ctot;
  // SYNC_ACK reuse: the SYNC classify also classifies the reverse direction of every
  // local message (its SYNC_ACK compares the same two rows with the roles swapped)
  uint2* rev_chunk;     // per (SYNC message, chunk): reverse (pool base, complex count)
  uint32_t* rev_total;  // per SYNC message: reverse complex count
  uint32_t* row_mod;    // per owned viewer: tick whose SYNC merge may have changed the row
  uint32_t* senders;    // local indices of this round's senders with live gossips
  uint32_t* pool;       // subjects whose record may change the receiver, chunk-ordered
  uint32_t pool_cap;
  uint32_t chunks;      // ceil(N / SYNC_CHUNK)
};

// Device-resident launch parameters.  Per-tick kernels receive only a pointer to these and the tick
// number instead of ~700 B of Ctx + Bufs by value: kernel arguments are read by dependent rounds of
// scalar loads that miss a cold scalar cache at every launch (~2 us each; measured 2-16 us of
// prologue per kernel), while this block sits in ordinary cached device memory.  The host uploads
// it only when a field changes (engine.hip, sync_params).
struct Params {
  Ctx c;   // T is taken from the kernel argument
  Ctx cs;  // the SYNC phase's context (its own list-insert counters)
  Bufs b;
};
__device__ __forceinline__ Ctx pctx(const Params* __restrict__ P, uint64_t T) {
  Ctx c = P->c;
  c.T = T;
  return c;
}
__device__ __forceinline__ Ctx pctx_sync(const Params* __restrict__ P, uint64_t T) {
  Ctx c = P->cs;
  c.T = T;
  return c;
}
#define KP const Params* __restrict__ P, uint64_t T

// ------------------------------------------------------------------------------- init
__global__ void k_init_rows(Ctx c, uint32_t n_initial) {
  const uint32_t conv_aux = A_IN_MEMBERS | A_ALIVE_EMITTED | A_HAS_METADATA;
  // the block witness starts from the converged row: ref = every initial member ALIVE at incarnation 0
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < c.n; s += gridDim.x * blockDim.x) {
    c.ref[s] = s < n_initial ? REC_IN_TABLE : 0u;
    c.dirty[s] = 0u;
  }
  for (uint32_t v = c.lo + blockIdx.x; v < c.lo + c.nl; v += gridDim.x) {
    uint32_t* r = rec_row(c, v);
    uint32_t* a = aux_row(c, v);
    const bool init = v < n_initial;
    for (uint32_t s = threadIdx.x; s < c.n; s += blockDim.x) {
      const bool in = init && s < n_initial;
      r[s] = in ? REC_IN_TABLE : 0u;  // ALIVE, incarnation 0
      a[s] = in ? (s == v ? A_IN_MEMBERS : conv_aux) : 0u;
    }
    // an initial row equals ref; a free slot's empty row differs at every initial member
    for (uint32_t blk = threadIdx.x; blk < c.blocks; blk += blockDim.x) {
      const uint32_t b0 = blk << BLK_SHIFT, b1 = min(c.n, b0 + (1u << BLK_SHIFT));
      const uint32_t in_blk = n_initial > b0 ? min(n_initial, b1) - b0 : 0u;
      c.bdiff[(size_t)(v - c.lo) * c.blocks + blk] = init ? 0u : in_blk;
    }
    if (threadIdx.x == 0) c.bnz[v - c.lo] = init ? 0u : (n_initial + (1u << BLK_SHIFT) - 1) >> BLK_SHIFT;
  }
}

// smallest tick t > after with t > start and (t - start) % period == 0: the next firing of a timer
// started at `start` (first fire one period after it)
__device__ inline uint32_t next_due(int64_t start, uint64_t after, uint32_t period) {
  const int64_t a = (int64_t)after > start ? (int64_t)after : start;
  return (uint32_t)(start + ((a - start) / (int64_t)period + 1) * (int64_t)period);
}

__device__ inline uint32_t fd_next_of(const Ctx& c, const MemberDev& m, uint64_t T) {
  uint32_t t = next_due(m.fd_start, T, c.P);
  if (m.ack_due > T && m.ack_due < t) t = (uint32_t)m.ack_due;
  if (m.relay_due > T && m.relay_due < t) t = (uint32_t)m.relay_due;
  return t;
}

// initial members: converged state, seeded Fisher-Yates ping / remote lists
__global__ void k_init_members(Ctx c, uint32_t n_initial, int32_t sync_stagger, int32_t timer_stagger) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.nl) return;
  const uint32_t v = c.lo + i;
  MemberDev m{};
  m.ack_target = NONE;
  m.relay_target = NONE;
  m.leave_gossiper = NONE;
  m.remote_idx = -1;
  if (v < n_initial) {
    m.joined = 1;
    m.table_size = n_initial;
    m.members_size = n_initial;
    uint32_t* pl = ping_list(c, v);
    uint32_t* rl = remote_list(c, v);
    uint32_t k = 0;
    for (uint32_t s = 0; s < n_initial; ++s)
      if (s != v) { pl[k] = s; rl[k] = s; ++k; }
    for (uint32_t i = k; i > 1; --i) {
      uint32_t j = next_int(draw_at(c, v, 0, SWIM_STREAM_INIT_PING, 0, i), i);
      uint32_t t = pl[i - 1]; pl[i - 1] = pl[j]; pl[j] = t;
    }
    for (uint32_t i = k; i > 1; --i) {
      uint32_t j = next_int(draw_at(c, v, 0, SWIM_STREAM_INIT_REMOTE, 0, i), i);
      uint32_t t = rl[i - 1]; rl[i - 1] = rl[j]; rl[j] = t;
    }
    m.ping_len = k;
    m.remote_len = k;
    m.remote_idx = 0;
    m.sync_on = 1;
    m.sync_start = sync_stagger ? -(int64_t)next_int(draw_at(c, v, 0, SWIM_STREAM_INIT_SYNC_PHASE, 0, 0), c.S) : 0;
    if (timer_stagger) {
      m.fd_start = -(int64_t)next_int(draw_at(c, v, 0, SWIM_STREAM_INIT_FD_PHASE, 0, 0), c.P);
      m.g_start = -(int64_t)next_int(draw_at(c, v, 0, SWIM_STREAM_INIT_GOSSIP_PHASE, 0, 0), c.G);
    }
  }
  c.mem[i] = m;
  c.gs[i] = GossipSched{next_due(m.g_start, c.T, c.G), 0u, 0u, 0u};
  c.fd_next[i] = m.joined ? fd_next_of(c, m, c.T) : NONE;
  c.sync_next[i] = m.sync_on ? next_due(m.sync_start, c.T, c.S) : NONE;
  c.mflag[i] = 0;
}

// ------------------------------------------------------------------------------- block scan helper
// exclusive scan of one uint32 per thread across the workgroup; returns the total in *total
template <int BLOCK>
__device__ inline uint32_t block_exclusive_scan(uint32_t x, uint32_t* s_wave, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < BLOCK / 64; ++w) { uint32_t t = s_wave[w]; s_wave[w] = acc; acc += t; }
    s_wave[BLOCK / 64] = acc;
  }
  __syncthreads();
  uint32_t r = s_wave[wave] + incl - x;
  *total = s_wave[BLOCK / 64];
  __syncthreads();
  return r;
}

// ------------------------------------------------------------------------------- start joins
// (the host has already set the replicated up[v] on every shard)
__global__ void k_start_joins(KP) {
  const Ctx c = pctx(P, T);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.nl) return;
  const uint32_t v = c.lo + i;
  MemberDev& m = c.mem[i];
  if (!m.join_pending) return;
  m.join_pending = 0;
  m.joined = 1;
  m.join_now = 1;
  m.init_wait = 1;
  m.init_pend = 0;
  c.pa_n[i] = 0;
  c.mflag[i] &= ~MF_PACK;
  m.init_last = (uint32_t)c.T;
  m.fd_start = (int64_t)c.T;
  m.g_start = (int64_t)c.T;
  c.gs[i].next = (uint32_t)c.T + c.G;
  cell_put(c, v, v, B_IN_TABLE | B_IN_MEMBERS);
  m.table_size = 1;
  m.members_size = 1;
  c.fd_next[i] = fd_next_of(c, m, c.T);
  c.mflag[i] |= MF_JOIN;
}

// ------------------------------------------------------------------------------- phase A
// onSuspicionTimeout (MembershipProtocolImpl.java:825-834) for every due (viewer, subject).
// A timer is queued by deadline bucket and by the 256-viewer block of its viewer, so the k_fd
// workgroup of that block fires it just before the block's FD steps (a per-viewer dependency: the
// timer touches only its viewer's state).  Entries of one viewer are independent (each touches only
// its own cell; counters are atomic), so the queue is processed entry-parallel; event order is
// canonicalised by minor = subject.
__device__ inline void timers_block(const Ctx& c, uint64_t T) {
  const uint32_t bucket = (uint32_t)(T & c.wheel_mask);
  const size_t q = (size_t)bucket * c.wheel_nq + blockIdx.x;
  uint32_t* qc = c.wheel_cnt + q;
  const uint32_t cnt = min(*qc, c.wheel_ptmax << c.wheel_pshift);
  const uint32_t pmask = (1u << c.wheel_pshift) - 1;
  uint32_t* pt = c.wheel_pt + q * c.wheel_ptmax;
  const uint32_t tmask = (uint32_t)(c.T & SWIM_DEADLINE_MASK);
  unsigned long long fired = 0;
  for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
    const uint32_t pid = pt[i >> c.wheel_pshift];
    if (pid >= c.wheel_pages) continue;  // never allocated (ERR_WHEEL is set)
    uint64_t* slot = c.wheel + ((size_t)pid << c.wheel_pshift) + (i & pmask);
    const uint64_t e = *slot;
    *slot = WHEEL_EMPTY;  // consumed: a recycled page holds no stale entry (schedule_timer may give up on a slot)
    const uint32_t v = (uint32_t)(e >> 32), s = (uint32_t)e;
    if (v - c.lo >= c.nl || !c.up[v]) continue;  // (WHEEL_EMPTY: a slot whose writer gave up, ERR_WHEEL)
    uint32_t* ap = aux_row(c, v) + s;
    uint32_t old = *ap;
    bool claimed = false;
    while ((old & A_HAS_TIMER) && (old >> 4) == tmask) {
      const uint32_t prev = atomicCAS(ap, old, old & ~A_HAS_TIMER);
      if (prev == old) { claimed = true; break; }
      old = prev;
    }
    if (!claimed) continue;
    fired++;
    const uint32_t r = rec_row(c, v)[s];
    if (r_in_table(r)) update_membership(c, v, s, SWIM_DEAD, r_inc(r), R_TIMEOUT, SWIM_PHASE_TIMERS);
  }
  wave_stat_add(c, ST_TIMERS_FIRED, fired);
  __syncthreads();  // the block's DEAD updates (lists to compact) are visible to every thread
  if (cnt) {  // the queue's pages are reusable from the next tick (k_end_tick)
    const uint32_t np = (cnt + pmask) >> c.wheel_pshift;
    for (uint32_t g = threadIdx.x; g < np; g += blockDim.x) {
      const uint32_t pid = pt[g];
      pt[g] = NONE;
      if (pid < c.wheel_pages) c.wheel_freed[atomicAdd(&c.wheel_ctl->freed, 1u)] = pid;
    }
    if (threadIdx.x == 0) *qc = 0;
  }
}

// REMOVED -> pingMembers.remove / remoteMembers.remove (FailureDetectorImpl.java:323-333,
// GossipProtocolImpl.java:240-251): both lists hold exactly the viewer's other `members`, so the
// removal is a stable compaction keeping in_members entries.
template <int BLOCK>
__device__ void compact_list(const Ctx& c, uint32_t v, uint32_t* list, uint32_t& len) {
  __shared__ uint32_t s_wave[BLOCK / 64 + 1];
  const uint32_t* a = aux_row(c, v);
  uint32_t out = 0;
  for (uint32_t base = 0; base < len; base += BLOCK) {
    uint32_t i = base + threadIdx.x;
    uint32_t val = 0, keep = 0;
    if (i < len) { val = list[i]; keep = (a[val] & A_IN_MEMBERS) ? 1u : 0u; }
    uint32_t total;
    uint32_t pos = block_exclusive_scan<BLOCK>(keep, s_wave, &total);
    if (keep) list[out + pos] = val;
    out += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) len = out;
  __syncthreads();
}

// ArrayList.remove(Object): the first x, later elements shift down one place
__device__ inline void list_remove(uint32_t* list, uint32_t& len, uint32_t x) {
  uint32_t j = 0;
  while (j < len && list[j] != x) ++j;
  if (j == len) return;
  for (; j + 1 < len; ++j) list[j] = list[j + 1];
  len--;
}

// ------------------------------------------------------------------------------- phase B
// publishPingResult (FailureDetectorImpl.java:377-380) -> onFailureDetectorEvent (:418-449)
__device__ inline void publish_fd(const Ctx& c, uint32_t v, uint32_t t, uint32_t status, unsigned long long& nev) {
  nev++;
  MemberDev& m = mem(c, v);
  if (c.record_fd)
    emit(c, v, t, SWIM_EV_FD_ALIVE + (status == SWIM_ALIVE ? 0 : status == SWIM_SUSPECT ? 1 : 2), SWIM_PHASE_FD,
         m.ev_minor++);
  const uint64_t cell = cell_get(c, v, t);
  if (!c_has(cell, B_IN_TABLE)) return;
  if (c_status(cell) == status) return;
  if (status == SWIM_ALIVE) {
    if (m.fd_sync_cnt >= FD_SYNC_MAX) { set_err(c, ERR_FDSYNC); return; }
    c.fd_sync[(size_t)(v - c.lo) * FD_SYNC_MAX + m.fd_sync_cnt++] = t;
    c.mflag[v - c.lo] |= MF_FDSYNC;
    return;
  }
  update_membership(c, v, t, status, c_inc(cell), R_FD_EVENT, SWIM_PHASE_FD);
  if (status == SWIM_DEAD && !(aux_row(c, v)[t] & A_IN_MEMBERS)) {
    // a DEST_GONE ack removed t inside the FD step: pingMembers / remoteMembers.remove(t) now
    // (FailureDetectorImpl.java:323-333, GossipProtocolImpl.java:240-251), before the member's
    // doPing picks its target; the serial shift is ArrayList.remove (rare: one per restart seen)
    MemberDev& m = mem(c, v);
    list_remove(ping_list(c, v), m.ping_len, t);
    list_remove(remote_list(c, v), m.remote_len, t);
  }
}

// selectPingReqMembers (:363-375) as a forward partial Fisher-Yates over pingMembers \ {target}
__device__ inline uint32_t select_relays(const Ctx& c, uint32_t v, uint32_t t, uint32_t* out) {
  const int32_t k = c.ping_req_members;
  if (k <= 0) return 0;
  const MemberDev& m = mem(c, v);
  const uint32_t* pl = ping_list(c, v);
  int64_t pos = -1;
  for (uint32_t i = 0; i < m.ping_len; ++i)
    if (pl[i] == t) { pos = i; break; }
  const uint32_t cnt = m.ping_len - (pos >= 0 ? 1u : 0u);
  if (cnt == 0) return 0;
  const uint32_t r = min((uint32_t)k, cnt);
  uint32_t swp_pos[32], swp_val[32];
  uint32_t nsw = 0;
  for (uint32_t i = 0; i < r; ++i) {
    uint32_t j = i + next_int(draw(c, v, SWIM_STREAM_RELAY_SELECT, i, 0), cnt - i);
    uint32_t vi = i, vj = j;
    for (uint32_t q = 0; q < nsw; ++q) { if (swp_pos[q] == i) vi = swp_val[q]; if (swp_pos[q] == j) vj = swp_val[q]; }
    // set(i, vj); set(j, vi)
    bool fi = false, fj = false;
    for (uint32_t q = 0; q < nsw; ++q) {
      if (swp_pos[q] == i) { swp_val[q] = vj; fi = true; }
      else if (swp_pos[q] == j) { swp_val[q] = vi; fj = true; }
    }
    if (!fi) { swp_pos[nsw] = i; swp_val[nsw] = vj; nsw++; }
    if (!fj && j != i) { swp_pos[nsw] = j; swp_val[nsw] = vi; nsw++; }
    if (j == i) { /* set(i, vj) then set(j, vi) with vi == vj: already consistent */ }
    out[i] = (pos >= 0 && (int64_t)vj >= pos) ? pl[vj + 1] : pl[vj];
  }
  return r;
}

// doPing's error branch (:153-170) + doPingReq (:173-210); the relays share the ping's correlation
// id, so the first relayed ack to reach the issuer completes every pending relay request.  With
// message delay the first message carrying the cid decides: the earliest relayed ack (ties: lowest
// relay) or a late ack of the direct ping (`late` = 1 + its arrival in ticks after the ping-req went
// out), if the issuer's inbound filter passes its sender; none before the relay timeout: SUSPECT.
// Every message goes to an address (dst): a relay's transit ping reaches whoever listens at t's
// address, whose onPing answers DEST_GONE when it is not t (:227-259); every ack carries that back
// (onTransitPingAck :291-315) and computeMemberStatus turns it into DEAD (:382-404).
__device__ inline void ping_req(const Ctx& c, uint32_t v, uint32_t t, unsigned long long& nev,
                                unsigned long long& nreq, uint32_t late = 0, bool late_gone = false) {
  uint32_t relays[16];
  uint32_t nr = select_relays(c, v, t, relays);
  if (nr == 0) { publish_fd(c, v, t, SWIM_SUSPECT, nev); return; }
  nreq++;
  const uint32_t d = dst(c, t);
  uint32_t pending_mask = 0, npend = 0;
  for (uint32_t j = 0; j < nr; ++j) {
    if (out_fail(c, v, dst(c, relays[j]), v, SWIM_STREAM_PINGREQ_OUT, j, 0)) publish_fd(c, v, t, SWIM_SUSPECT, nev);
    else { pending_mask |= 1u << j; npend++; }
  }
  if (npend == 0) return;
  uint32_t best = NONE, first = NONE;  // arrival (ticks from now) and sender of the first ack
  bool first_gone = d != t;
  for (uint32_t j = 0; j < nr; ++j) {
    if (!(pending_mask & (1u << j))) continue;
    uint32_t r = dst(c, relays[j]);
    if (in_pass(c, r, v) && !out_fail(c, r, d, v, SWIM_STREAM_TRANSIT_PING_OUT, j, 0) &&
        in_pass(c, d, r) && !out_fail(c, d, r, v, SWIM_STREAM_TRANSIT_ACK_OUT, j, 0) &&
        in_pass(c, r, d) && !out_fail(c, r, v, v, SWIM_STREAM_RELAY_ACK_OUT, j, 0)) {
      const uint32_t at = delay_ticks(c, v, r, v, SWIM_STREAM_PINGREQ_DELAY, j, 0) +
                          delay_ticks(c, r, d, v, SWIM_STREAM_TRANSIT_PING_DELAY, j, 0) +
                          delay_ticks(c, d, r, v, SWIM_STREAM_TRANSIT_ACK_DELAY, j, 0) +
                          delay_ticks(c, r, v, v, SWIM_STREAM_RELAY_ACK_DELAY, j, 0);
      if (at < best) { best = at; first = r; }
      if (!c.delay_on) break;  // every arrival is 0: the lowest relay
    }
  }
  if (late && late - 1 < best) { best = late - 1; first = d; first_gone = late_gone; }
  MemberDev& m = mem(c, v);
  // the issuer's inbound filter meets the first ack when it arrives (NetworkEmulatorTransport
  // .requestResponse :72-74): now, or at relay_due (fd_member)
  if (first != NONE && best < c.relay_ticks && (best > 0 || in_pass(c, v, first))) {
    if (best == 0) {
      for (uint32_t i = 0; i < npend; ++i) publish_fd(c, v, t, first_gone ? SWIM_DEAD : SWIM_ALIVE, nev);
      return;
    }
    m.relay_due = c.T + best;  // the first ack arrives then and completes every pending relay request
    m.relay_ok = 1;
    m.relay_gone = first_gone ? 1 : 0;
    m.relay_first = first;
    m.relay_to = c.T + c.relay_ticks;
  } else {
    m.relay_due = c.T + c.relay_ticks;
    m.relay_ok = 0;
  }
  m.relay_target = t;
  m.relay_pending = npend;
}

__device__ inline void fd_member(const Ctx& c, uint32_t v, unsigned long long& nev, unsigned long long& nreq,
                                 unsigned long long& npings) {
  MemberDev& m = mem(c, v);
  if (!c.up[v]) return;  // a stopped member's timers stop; a join restarts them (fd_next)
  const bool due = (int64_t)c.T > m.fd_start && ((int64_t)c.T - m.fd_start) % c.P == 0;
  c.fd_next[v - c.lo] = fd_next_of(c, m, c.T);  // ack / relay timeouts set below are > T
  if (!due && m.relay_due != c.T && m.ack_due != c.T) return;
  m.ev_minor = 0;
  if (m.relay_due == c.T && m.relay_ok && !in_pass(c, v, m.relay_first)) {
    // the first relayed ack arrives and the inbound filter drops it: no pending relay request
    // completes (each took the first message with the cid), they time out
    m.relay_ok = 0;
    m.relay_due = m.relay_to;
  }
  if (m.ack_due == c.T && m.ack_ok && !in_pass(c, v, dst(c, m.ack_target))) {
    m.ack_ok = 0;  // the delayed ack is dropped on arrival: the ping waits for its timeout
    m.ack_due = m.ack_to;
  }
  if (m.relay_due == c.T) {  // relayed acks arrive (:190-199) or the relay timeouts (:200-209)
    uint32_t t = m.relay_target, k = m.relay_pending;
    m.relay_due = 0;
    const uint32_t ok_status = m.relay_gone ? SWIM_DEAD : SWIM_ALIVE;
    for (uint32_t i = 0; i < k; ++i) publish_fd(c, v, t, m.relay_ok ? ok_status : SWIM_SUSPECT, nev);
  }
  if (m.ack_due == c.T) {  // the delayed ack arrives, or pingTimeout elapsed
    uint32_t t = m.ack_target;
    m.ack_due = 0;
    if (m.ack_ok) publish_fd(c, v, t, m.ack_gone ? SWIM_DEAD : SWIM_ALIVE, nev);
    else ping_req(c, v, t, nev, nreq, m.ack_late, m.ack_gone != 0);
  }
  if (due) {  // doPing (:126-171), selectPingMember (:352-361)
    m.fd_period++;
    if (m.ping_len > 0) {
      uint32_t* pl = ping_list(c, v);
      if (m.ping_cursor >= m.ping_len) {
        m.ping_cursor = 0;
        shuffle_list(c, v, pl, m.ping_len, SWIM_STREAM_FD_SHUFFLE);
      }
      uint32_t t = pl[m.ping_cursor++];
      npings++;
      const uint32_t d = dst(c, t);  // whoever listens at t's address now
      if (out_fail(c, v, d, v, SWIM_STREAM_PING_OUT, 0, 0)) {
        ping_req(c, v, t, nev, nreq);
      } else {
        // onPing answers DEST_OK, or DEST_GONE from another member at t's address (:227-259) ->
        // computeMemberStatus ALIVE / DEAD (:382-404); the round trip takes both messages' delays
        const bool acked = in_pass(c, d, v) && !out_fail(c, d, v, v, SWIM_STREAM_ACK_OUT, 0, 0);
        const uint32_t rtt = acked ? delay_ticks(c, v, d, v, SWIM_STREAM_PING_DELAY, 0, 0) +
                                         delay_ticks(c, d, v, v, SWIM_STREAM_ACK_DELAY, 0, 0)
                                   : 0u;
        m.ack_gone = d != t ? 1 : 0;
        if (acked && rtt == 0 && in_pass(c, v, d)) {
          publish_fd(c, v, t, d != t ? SWIM_DEAD : SWIM_ALIVE, nev);
        } else {
          // a delayed ack meets the issuer's inbound filter when it arrives (above)
          m.ack_target = t;
          m.ack_ok = acked && rtt > 0 && rtt < c.to_ticks;
          m.ack_due = c.T + (m.ack_ok ? rtt : c.to_ticks);
          m.ack_to = c.T + c.to_ticks;
          m.ack_late = acked && rtt >= c.to_ticks ? rtt - c.to_ticks + 1 : 0;
        }
      }
    }
  }
  c.fd_next[v - c.lo] = fd_next_of(c, m, c.T);
}

// ------------------------------------------------------------------------------- phase C

// checkGossipSegmentation (GossipProtocolImpl.java:217-236); only launched when the threshold is
// below the inline interval capacity (otherwise a clear can never trigger).

// Gossip inboxes are paged: receiver i's k-th message of the round lives in page
// pg_tab[i][k / 64], slot k % 64; pages come from a per-tick bump pool, so emit and k_recv_msgs write
// every message straight into its receiver's inbox (no grouping pass) and the deliverer hands the
// pages back by resetting the receiver's page table.  Exactly one writer allocates each page: the
// one whose reserved slots include the page's first slot; a writer whose slots start inside a page
// waits for that page (its first slot was reserved earlier, by a writer that allocates it without
// waiting).  Writers allocate before they wait, so a wave never waits on one of its own lanes.
// A receiver's FIRST page is its own, pool page i, fixed for the engine's life (pg_tab[i][0] = i,
// never handed back): a storm's inboxes mostly fit one page, so most writers neither allocate nor
// wait, and the small-inbox delivery needs no page-table load; the bump pool starts after them.
constexpr uint32_t PG_FAILED = 0xfffffffeu;  // the pool ran dry: releases the page's waiters
__device__ inline uint32_t inbox_page_alloc(const Ctx& c, const Bufs& b, uint32_t i, uint32_t pg) {
  if (pg == 0) return i;
  if (pg >= b.pg_max) { set_err(c, ERR_INBOX); return NONE; }
  uint32_t np = c.nl + atomicAdd(&b.k->pg_cursor, 1u);
  if (np >= b.pg_cap) { set_err(c, ERR_PAGES); np = PG_FAILED; }
  __atomic_store_n(b.pg_tab + (size_t)i * b.pg_max + pg, np, __ATOMIC_RELAXED);
  return np == PG_FAILED ? NONE : np;
}
__device__ inline uint32_t inbox_page_wait(const Ctx& c, const Bufs& b, uint32_t i, uint32_t pg) {
  if (pg == 0) return i;
  if (pg >= b.pg_max) { set_err(c, ERR_INBOX); return NONE; }
  const uint32_t* e = b.pg_tab + (size_t)i * b.pg_max + pg;
  for (uint32_t it = 0; it < (1u << 20); ++it) {
    const uint32_t v = __atomic_load_n(e, __ATOMIC_RELAXED);
    if (v != NONE) return v == PG_FAILED ? NONE : v;
    __builtin_amdgcn_s_sleep(2);
  }
  set_err(c, ERR_PAGES);  // bounded: never reached while the page's allocator runs
  return NONE;
}
// the receiver's inbox crossed the per-thread delivery limit: the wave-parallel path takes it
__device__ __forceinline__ void big_mark(const Bufs& b, uint32_t i, uint64_t T) {
  b.big_list[atomicAdd(&b.k->big_cnt, 1u)] = i;
  b.big_tick[i] = (uint32_t)T;
}
__device__ __forceinline__ void wave_order() {
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}
// LDS writes of one lane made visible to the wave's other lanes without waiting for the wave's
// outstanding global loads (s_waitcnt lgkmcnt(0) only: a wave's LDS operations complete in order)
__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

// a GOSSIP_REQ for a receiver owned by this shard joins the receiver's inbox (every lane of the wave
// calls it: `valid` masks the lanes without a message); in the inbox, `to` holds the message's age
__device__ inline void deliver_local_msg(const Ctx& c, const Bufs& b, GMsgFull msg, bool valid, uint32_t age) {
  const uint32_t i = msg.to - c.lo;
  msg.to = age;
  uint32_t s = 0, pid = NONE;
  if (valid) {
    s = atomicAdd(&b.msg_cnt[i], 1u);
    if (s == b.wave_min) big_mark(b, i, c.T);
    if ((s & 63) == 0) pid = inbox_page_alloc(c, b, i, s >> 6);
  }
  wave_order();
  if (valid && (s & 63) != 0) pid = inbox_page_wait(c, b, i, s >> 6);
  if (valid && pid != NONE) {
    b.pg_msgs[(size_t)pid * 64 + (s & 63)] = msg;
    b.k->msg_total = 1u;  // "some inbox is non-empty" (k_gossip_deliver's early exit)
  }
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {  // lane 0 gets the wave's sum
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_down(x, d, 64);
  return x;
}
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// doSpreadGossip (:141-184), wave-parallel.  Each wave owns the senders wid, wid + nw, ... and
// first checks up to 64 of them at once (lane l: sender base + l * nw): every due sender advances
// its period (:143); a sender with live gossips then gets the whole wave: lane 0 selects the
// targets (:322-343), the (target, slab position) pairs of selectGossipsToSend (:311-320) are
// spread over the lanes — loss draws and receiver-collector probes of 64 pairs in flight together,
// one inbox atomic per (target, pass) — and the same pass over the slab also sweeps it (:158-164,
// order preserving) and checks the futures.
constexpr int EMIT_WAVES = 4;
// profiling builds: the emit kernel's part times and counts, per wave in registers (added to g_dbg
// 16..23 once per wave at the end of the kernel: no contended atomic per sender or per pass)
struct EmitProf {
  unsigned long long t_setup = 0, t_pass = 0, t_win = 0, t_mat = 0, n_all = 0, n_win = 0, n_mat = 0, n_snd = 0;
  unsigned long long t_sel = 0, t_tgt = 0;  // setup parts: target selection, per-target words
};
// A sender's round setup loaded ahead, for all of a wave's senders at once (lane j: its j-th sender):
// the targets selectGossipMembers takes without a reshuffle (remoteMembers[idx .. idx + F), every
// member on its own address) and their per-target words.  ok = 0: the sender selects in line.
constexpr uint32_t PRE_F = 4;  // fanouts up to this are taken ahead
struct SenderPre {
  uint32_t ok;
  uint32_t rlen;       // remoteMembers.size()
  int32_t idx;         // remoteMembersIndex
  uint32_t fut;        // a graceful leave or an own user gossip is pending (futures to check)
  uint32_t pw;         // the member holds PAcks (some may wait on its LEAVING gossips)
  uint32_t t[PRE_F];   // targets
  uint32_t tw[PRE_F];  // up | inbound-passes << 1 | v's outbound loss towards it << 2
  uint32_t clr[PRE_F]; // its collectors' last clear tick (owned, or the peer's: receipt filter), else ~0
};
// the last clear tick of target t's collectors, as the receipt check compares it: t's own shard's, or
// (cross-shard receipt filter) the peer's; ~0 = no receipt bit of t is trusted
__device__ __forceinline__ uint32_t target_clr(const Ctx& c, const Bufs& b, uint32_t t) {
  if (owned(c, t)) return c.clr_tick[t - c.lo];
  if (!b.rfilter) return 0xffffffffu;
  const uint32_t p = t / c.sz;
  return b.peers->clr_tick[p][t - p * c.sz];
}
__device__ __forceinline__ void sender_pre_load(const Ctx& c, const Bufs& b, uint32_t i, SenderPre& sp) {
  sp.ok = 0;
  const MemberDev& m = c.mem[i];
  const uint32_t rlen = m.remote_len;
  const int32_t idx = m.remote_idx;
  sp.rlen = rlen;
  sp.idx = idx;
  sp.fut = (m.leave_pending || m.user_live) ? 1u : 0u;
  sp.pw = (c.mflag[i] & MF_PACK) ? 1u : 0u;
  const uint32_t F = (uint32_t)c.fanout;
  if (F > PRE_F || c.route) return;
  if (rlen < F || idx < 0 || (uint32_t)idx + F > rlen) return;
  const uint32_t v = c.lo + i;
  const uint32_t* rl = remote_list(c, v) + idx;
#pragma unroll
  for (uint32_t q = 0; q < PRE_F; ++q) sp.t[q] = q < F ? rl[q] : 0u;
#pragma unroll
  for (uint32_t q = 0; q < PRE_F; ++q) {
    if (q >= F) continue;
    const uint32_t t = sp.t[q];
    sp.tw[q] = (c.up[t] ? 1u : 0u) | (in_pass(c, t, v) ? 2u : 0u) | ((uint32_t)out_loss(c, v, t) << 2);
    sp.clr[q] = target_clr(c, b, t);
  }
  sp.ok = 1;
}
__device__ __forceinline__ uint32_t pick4(const uint32_t (&a)[PRE_F], uint32_t q) {
  return q == 0 ? a[0] : q == 1 ? a[1] : q == 2 ? a[2] : a[3];
}
__device__ __forceinline__ SenderPre sender_pre_from(const SenderPre& x, int j) {
  SenderPre sp;
  sp.ok = rdlane(x.ok, j);
  sp.rlen = rdlane(x.rlen, j);
  sp.idx = (int32_t)rdlane((uint32_t)x.idx, j);
  sp.fut = rdlane(x.fut, j);
  sp.pw = rdlane(x.pw, j);
#pragma unroll
  for (uint32_t q = 0; q < PRE_F; ++q) {
    sp.t[q] = rdlane(x.t[q], j);
    sp.tw[q] = rdlane(x.tw[q], j);
    sp.clr[q] = rdlane(x.clr[q], j);
  }
  return sp;
}

__device__ __forceinline__ unsigned long long gossip_emit_sender(const Ctx& c, const Bufs& b, uint32_t v, uint64_t period,
                                                        uint32_t glen, uint32_t gbase, uint32_t lane, uint32_t* s_t,
                                                        unsigned long long& nmat, unsigned long long& nexam,
                                                        EmitProf& ep,
                                                        const SenderPre& sp, const GossipHot h_head,
                                                        const GossipHot h_tail) {
  PPROF_T0(te0);
#ifdef SWIM_PHASE_PROF
  ep.n_snd++;
  unsigned long long& np_all = ep.n_all;
  unsigned long long& np_win = ep.n_win;
  unsigned long long& np_mat = ep.n_mat;
  unsigned long long& t_win = ep.t_win;
  unsigned long long& t_mat = ep.t_mat;
#endif
  MemberDev& m = mem(c, v);
  const SlabRef slab = slab_of(c, v, gbase);
  // both ends of the slab (see below) were loaded by the caller during the previous sender: the first
  // 64 states and the last 64
  const uint32_t tail0 = glen > 64 ? glen - 64 : 0u;
  const uint32_t rlen = sp.rlen;
  const uint32_t F = (uint32_t)c.fanout;
  if (sp.ok) {  // the targets and their words were loaded ahead (no reshuffle, no shared address)
    if (lane == 0) {
      s_t[0] = F;
      s_t[49] = 0;
      m.remote_idx = sp.idx + (int32_t)F;
    }
    if (lane < F) {  // (register arrays read through selects, never a runtime index: no scratch)
      const uint32_t t = pick4(sp.t, lane), tw = pick4(sp.tw, lane);
      s_t[1 + lane] = t;
      s_t[17 + lane] = t;
      s_t[33 + lane] = lane;
      s_t[50 + lane] = tw & 3u;
      s_t[66 + lane] = tw >> 2;
      s_t[82 + lane] = pick4(sp.clr, lane);
    }
  } else if (lane == 0) {  // selectGossipMembers (:322-343)
    uint32_t* rl = remote_list(c, v);
    uint32_t nt = 0;
    if (rlen < F) {
      for (uint32_t i = 0; i < rlen; ++i) s_t[1 + nt++] = rl[i];
    } else {
      if (m.remote_idx < 0 || (uint32_t)m.remote_idx + F > rlen) {
        shuffle_list(c, v, rl, rlen, SWIM_STREAM_GOSSIP_SHUFFLE);
        m.remote_idx = 0;
      }
      for (uint32_t i = 0; i < F; ++i) s_t[1 + nt++] = rl[m.remote_idx + i];
      m.remote_idx += (int32_t)F;
    }
    s_t[0] = nt;
    // s_t[1 + j]: the member that receives what is sent to target j's address; s_t[17 + j]: target j;
    // s_t[33 + j]: the first target with the same receiver (an old member and the member restarted
    // on its address are both targets); s_t[49]: some target shares its receiver
    uint32_t alias = 0;
    for (uint32_t j = 0; j < nt; ++j) {
      s_t[17 + j] = s_t[1 + j];
      s_t[1 + j] = dst(c, s_t[1 + j]);
      uint32_t j0 = 0;
      while (s_t[1 + j0] != s_t[1 + j]) ++j0;
      s_t[33 + j] = j0;
      alias |= j0 != j ? 1u : 0u;
    }
    s_t[49] = alias;
  }
  lds_order();
  PPROF_ACC(ep.t_sel, te0);
  PPROF_T0(te_t);
  const uint32_t nt = s_t[0];
  // what depends on the target only, once per round instead of once per (target, gossip): whether
  // it is up (s_t[50 + j]; bit 1: its inbound filter passes v now — a delayed message meets the filter
  // when it arrives, k_dq_release), v's outbound loss towards it (s_t[66 + j]), the tick its
  // collectors were last cleared (s_t[82 + j]; receipt bits older than that are void)
  if (!sp.ok && lane < nt) {
    const uint32_t t = s_t[1 + lane];
    s_t[50 + lane] = (c.up[t] ? 1u : 0u) | (in_pass(c, t, v) ? 2u : 0u);
    s_t[66 + lane] = (uint32_t)out_loss(c, v, t);
    s_t[82 + lane] = target_clr(c, b, t);
  }
  lds_order();
  PPROF_ACC(ep.t_tgt, te_t);
  const uint64_t spread = (uint64_t)(c.repeat_mult * ceil_log2(rlen + 1));
  const uint64_t sweep = 2 * (spread + 1);
  const bool leaving = sp.fut && m.leave_pending != 0;
  unsigned long long nmsg = 0;
  uint32_t pseq = 0;  // lane j < nt: messages materialised to target j so far (GMsgFull.pseq)
  bool done = false;
  // Infection periods grow along the slab (every state is appended with the current period), so the
  // states a round must look at are ranges found from the ends: (1) the swept prefix, sweep
  // (:158-164, :350-358): period > infectionPeriod + periodsToSweep; (2) the in-window suffix
  // (:145-151, selectGossipsToSend): infectionPeriod + periodsToSpread >= period.  The states between
  // matter only to the futures (:167-180, :360-368) — a graceful leave's, or a user gossip's
  // spread() of this member — and are read only while one is pending.
  uint32_t lead = 0;  // (1): the first state kept
  for (uint32_t p0 = 0; p0 < glen; p0 += 64) {
    const uint32_t p = p0 + lane;
    bool sw = false;
    GossipHot h{};
    if (p < glen) {
      h = p0 == 0 ? h_head : slab.H(p);
      sw = period > (uint64_t)h.inf_period() + sweep;
    }
    // its infected overflow goes too: one lane at a time (inf_erase moves entries of the table)
    for (uint64_t dm = __ballot(sw && h.more()); dm; dm &= dm - 1) {
      if (lane == (uint32_t)__ffsll((unsigned long long)dm) - 1) slab.drop_more(h.gossiper, h.seq);
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
    }
    const uint64_t km = __ballot(p < glen && !sw);
    if (km) {
      lead = p0 + (uint32_t)__ffsll((unsigned long long)km) - 1;
      break;
    }
    lead = min(p0 + 64, glen);
  }
  uint32_t wst = glen;  // (2): the first in-window state (a swept state is out of the window too)
  for (uint32_t e0 = glen; e0 > lead;) {
    const bool last = e0 == glen;
    const uint32_t s0 = last ? tail0 : (e0 - lead > 64 ? e0 - 64 : lead);
    const uint32_t p = s0 + lane;
    bool out = false;
    if (p < e0) {
      const uint32_t per_st = last ? (glen > 64 ? h_tail.per_st : h_head.per_st) : slab.H(p).per_st;
      out = !((uint64_t)(per_st & PER_MASK) + spread >= period);
    }
    const uint64_t om = __ballot(out);
    if (om) {
      wst = max(lead, s0 + (64u - (uint32_t)__clzll((unsigned long long)om)));
      break;
    }
    wst = max(lead, s0);
    e0 = s0;
  }
  const uint32_t first = sp.fut ? lead : wst;
  nexam += lead + (glen > first ? glen - first : 0u);  // hot bytes read: the swept prefix and the passes
  // lane = slab position: one GossipState read serves all nt targets, whose loss draws and
  // receiver checks are independent (issued together); messages keep the (target, position) keys.
  // A pass reads the 16 hot bytes of each state; the 8 cold ones only where a message is
  // materialised (the infected overflow only for a state that has one).  The slab is a ring: the
  // sweep drops the prefix by advancing its base after the round, so nothing moves.
  // the next pass's hot bytes are loaded while this pass runs
  GossipHot hn{};
  if (first >= tail0) {  // the first pass lies in the tail already loaded: moved across lanes
    const bool tl = glen > 64;
    const int from = (int)(first - tail0 + lane) & 63;
    hn.gossiper = __shfl(tl ? h_tail.gossiper : h_head.gossiper, from, 64);
    hn.seq = __shfl(tl ? h_tail.seq : h_head.seq, from, 64);
    hn.per_st = __shfl(tl ? h_tail.per_st : h_head.per_st, from, 64);
    hn.inf0 = __shfl(tl ? h_tail.inf0 : h_head.inf0, from, 64);
  } else if (first + lane < glen) {
    hn = slab.Hg(first + lane);
  }
  uint32_t sinkw = 0;  // the next pass's receipt-slot lines, warmed at the end of this one
  PPROF_ACC(ep.t_setup, te0);
  PPROF_T0(te1);
  for (uint32_t p0 = first; p0 < glen; p0 += 64) {
#ifdef SWIM_PHASE_PROF
    np_all++;
#endif
    const uint32_t p = p0 + lane;
    const GossipHot h = hn;
    if (p + 64 < glen) hn = slab.Hg(p + 64);  // (a global load: the pass's LDS waits do not wait for it)
    bool win = false, keep = false;
    if (p < glen) {
      win = (uint64_t)h.inf_period() + spread >= period;
      keep = true;  // (p >= lead)
    }
    // futures: the graceful-leave future stops the member at the end of the tick; a user gossip's
    // spread() completes (this round's copies carry the status read above)
    bool changed = false;
    if (keep && period > (uint64_t)h.inf_period() + spread) {
      if (leaving && h.gossiper == m.leave_gossiper && h.seq == (uint32_t)m.leave_seq) done = true;
      if (h.status() == SWIM_GOSSIP_USER && h.gossiper == v) {
        changed = true;
        emit(c, v, v, SWIM_EV_SPREAD_DONE, SWIM_PHASE_GOSSIP, 0x80000000u | (h.seq & 0x7fffffffu), slab.C(p).subject);
      }
    }
    {
      const uint32_t nch = (uint32_t)__popcll(__ballot(changed));
      if (lane == 0 && nch) m.user_live -= nch;
    }
    uint32_t matb = 0;  // bit j: a message to target j is materialised
    uint32_t subj = 0;
    int32_t inc = 0;
    bool have_cold = false;
    auto load_cold = [&]() {
      if (!have_cold) {
        const GossipCold k = slab.C(p);
        subj = k.subject;
        inc = k.inc;
        have_cold = true;
      }
    };
    PPROF_T0(te2);
    if (__ballot(win)) {
#ifdef SWIM_PHASE_PROF
      np_win++;
#endif
      // the gossip's receipt-bitmap slot serves every target (one load per gossip)
      uint64_t key = 0;
      uint32_t sl = 0;
      GSlot gs{};
      if (win) {
        key = gkey(h.gossiper, h.seq);
        sl = gslot_of(key);
        gs = c.gslot[sl];
      }
      const bool gs_ok = win && gs.key == key;
      // the first four targets' receipt words are loaded beside the slot (their addresses need only
      // the slot index, not its contents): one round trip where the check needs two.  A target on
      // another shard (cross-shard receipt filter) has its word, and its slot, in the peer's bitmaps
      auto rword = [&](uint32_t jj) -> uint32_t {
        const uint32_t t = s_t[1 + min(jj, nt - 1)];
        if (!(win && jj < nt)) return 0u;
        if (owned(c, t)) return c.gbits[rbit_word(t - c.lo, sl)];
        if (!b.rfilter) return 0u;
        const uint32_t p = t / c.sz;
        return b.peers->gbits[p][rbit_word(t - p * c.sz, sl)];
      };
      const uint32_t wb0 = rword(0), wb1 = rword(1), wb2 = rword(2), wb3 = rword(3);
      // GossipState.infected beyond its first member (rare: the overflow table, once per pass)
      uint32_t xinf[GINF - 1];
#pragma unroll
      for (int q = 0; q < GINF - 1; ++q) xinf[q] = NONE;
      if (win && h.more()) {
        const int32_t f = inf_find(slab.inf, slab.inf_mask, h.gossiper, h.seq);
        if (f >= 0)
#pragma unroll
          for (int q = 0; q < GINF - 1; ++q) xinf[q] = slab.inf[f].inf[q];
      }
      uint32_t probe = 0;  // bit j: target j's collector must be probed (its receipt bit does not answer)
      for (uint32_t j = 0; j < nt; ++j) {
        const uint32_t t = s_t[1 + j], tm = s_t[17 + j];
        bool infected = h.inf0 == tm;
#pragma unroll
        for (int q = 0; q < GINF - 1; ++q) infected |= xinf[q] == tm;
        const bool send = win && !infected;
        nmsg += send ? 1u : 0u;
        // delivered copies; a receiver on this shard that already holds the sequence id drops it
        // (its collector only grows until delivery), another shard flags it on arrival
        bool mat = send && (s_t[50 + j] & 1u) && !lost_k(c, (int32_t)s_t[66 + j], v, SWIM_STREAM_GOSSIP_OUT, j, p);
        // a delayed copy waits in the arrival tick's bucket (delivered whatever the receiver's
        // collector holds by then: a clear may come in between; its inbound filter applies then)
        const uint32_t k = mat ? delay_ticks(c, v, t, v, SWIM_STREAM_GOSSIP_DELAY, j, p) : 0u;
        if (!k && !(s_t[50 + j] & 2u)) mat = false;  // dropped by the receiver's inbound filter now
        if (k) {
          mat = false;
          load_cold();
          const uint32_t bk = (uint32_t)(c.T + k) & DQ_MASK;
          const uint32_t q = atomicAdd(&b.dq_cnt[bk], 1u);
          if (q < b.dq_bcap) {
            GMsgFull msg;
            msg.to = t; msg.from = v; msg.pos_dup = p; msg.pseq = (uint32_t)c.T;  // (the sending tick)
            msg.set_gossip(h.gossiper, h.seq, subj, h.status(), inc);
            b.dq[(size_t)bk * b.dq_bcap + q] = msg;
          } else {
            set_err(c, ERR_DELAY);
          }
        }
        if (mat && owned(c, t)) {
          // exact: does t's collector hold (gossiper, seq)?  The receipt bit answers without the
          // collector probe when it is set and trustworthy (set after the slot's claim, and no
          // collector of t was cleared since the claim); else the collector is probed below, the
          // targets' probes in one batch
          const uint32_t i = t - c.lo;
          const uint32_t word = j == 0 ? wb0 : j == 1 ? wb1 : j == 2 ? wb2 : j == 3 ? wb3
                                                 : c.gbits[rbit_word(i, sl)];
          const bool known = gs_ok && s_t[82 + j] < gs.tick && ((word >> (sl & 31)) & 1u);
          if (known) mat = false;
          else probe |= 1u << j;
        } else if (mat && b.rfilter) {
          // cross-shard receipt filter: the same test against the receiver's shard's slot and bit
          // (every shard's tick-T timers and segmentation clears precede every emit of the tick, and
          // no delivery of the tick has run: the unsharded engine's view); without a trusted bit the
          // message is materialised (its collector is not probed: the receiver flags a duplicate)
          // (the peer's slot is loaded here, not beside the words: holding four slots' words
          // through the batch cost the unsharded kernel registers and spills)
          const uint32_t p = t / c.sz, i = t - p * c.sz;
          const uint32_t word = j == 0 ? wb0 : j == 1 ? wb1 : j == 2 ? wb2 : j == 3 ? wb3
                                                 : b.peers->gbits[p][rbit_word(i, sl)];
          if ((word >> (sl & 31)) & 1u) {
            const GSlot ps = b.peers->gslot[p][sl];
            if (ps.key == key && s_t[82 + j] < ps.tick) mat = false;
          }
        }
        matb |= (mat ? 1u : 0u) << j;
      }
      for (uint32_t j0 = 0; probe >> j0; j0 += 4) {  // the collector probes, four targets at a time
        const uint32_t need = (probe >> j0) & 0xfu;
        if (!need) continue;
        const uint32_t tg4[4] = {s_t[1 + min(j0, nt - 1)], s_t[1 + min(j0 + 1, nt - 1)], s_t[1 + min(j0 + 2, nt - 1)],
                                 s_t[1 + min(j0 + 3, nt - 1)]};
        matb &= ~(coll_known4(c, tg4, need, h.gossiper, h.seq) << j0);
      }
      if (s_t[49]) {
        // two targets at one address: their copies of this gossip are the same message to the same
        // receiver in the same round, and after the first the collector holds the sequence id
        // (onGossipReq :205 returns), so one copy is materialised, under the first such target,
        // which keeps the pair's pseq dense
        for (uint32_t j = 1; j < nt; ++j) {
          const uint32_t j0 = s_t[33 + j];
          if (j0 != j && ((matb >> j) & 1u)) matb = (matb & ~(1u << j)) | (1u << j0);
        }
      }
    }
    PPROF_ACC(t_win, te2);
    PPROF_T0(te3);
    if (__ballot(matb != 0)) {
#ifdef SWIM_PHASE_PROF
      np_mat++;
#endif
      if (matb) load_cold();
      // one inbox reservation per target present in this pass: lane j issues target j's atomic and
      // makes sure the (at most two) inbox pages of its slot range exist
      uint32_t cnt_mine = 0;
      for (uint32_t j = 0; j < nt; ++j) {
        const uint32_t cj = (uint32_t)__popcll(__ballot((matb >> j) & 1u));
        nmat += cj;  // wave-uniform
        if (lane == j) cnt_mine = cj;
      }
      uint32_t base = 0, pid0 = NONE, pid1 = NONE;
      const bool loc = lane < nt && cnt_mine && owned(c, s_t[1 + lane]);
      if (lane < nt && cnt_mine) {
        const uint32_t tj = s_t[1 + lane];
        if (loc) {
          const uint32_t i = tj - c.lo;
          base = atomicAdd(&b.msg_cnt[i], cnt_mine);
          if (base <= b.wave_min && base + cnt_mine > b.wave_min) big_mark(b, i, c.T);
          // pages whose first slot is ours: ours to allocate (first the second page, if any)
          if (((base + cnt_mine - 1) >> 6) != (base >> 6)) pid1 = inbox_page_alloc(c, b, i, (base >> 6) + 1);
          if ((base & 63) == 0) pid0 = inbox_page_alloc(c, b, i, base >> 6);
        } else {
          base = atomicAdd(&b.x->msg[owner(c, tj)], cnt_mine);
        }
      }
      wave_order();
      if (loc) {
        // our slots start inside a page another writer allocates
        if ((base & 63) != 0) pid0 = inbox_page_wait(c, b, s_t[1 + lane] - c.lo, base >> 6);
        if (((base + cnt_mine - 1) >> 6) == (base >> 6)) pid1 = pid0;
      }
      for (uint32_t j = 0; j < nt; ++j) {
        const bool mat = (matb >> j) & 1u;
        const uint64_t mk = __ballot(mat);
        if (!mk) continue;
        const uint32_t bj = rdlane(base, j), qj = rdlane(pseq, j);
        const uint32_t p0j = rdlane(pid0, j), p1j = rdlane(pid1, j);
        if (!mat) continue;
        const uint32_t pre = lanes_below(mk);
        const uint32_t t = s_t[1 + j];
        GMsgFull msg;
        msg.to = owned(c, t) ? 0u : t;  // in the inbox: age 0; for another shard: the receiver
        msg.from = v; msg.pos_dup = p; msg.pseq = qj + pre;
        msg.set_gossip(h.gossiper, h.seq, subj, h.status(), inc);
        if (owned(c, t)) {
          const uint32_t s = bj + pre;
          const uint32_t pid = (s >> 6) == (bj >> 6) ? p0j : p1j;
          if (pid != NONE) b.pg_msgs[(size_t)pid * 64 + (s & 63)] = msg;  // else inbox_page set the error bit
        } else {
          const uint32_t d = owner(c, t);
          if (bj + pre < b.tx_msg_cap) b.tx_msgs[(size_t)d * b.tx_msg_cap + bj + pre] = msg; else set_err(c, ERR_MSGS);
        }
      }
      pseq += cnt_mine;  // lane j: target j's messages so far this round
    }
    PPROF_ACC(t_mat, te3);
    // a state whose status changed is written back in place
    if (changed) {
      GossipHot hw = h;
      hw.per_st = (hw.per_st & ~(7u << PER_BITS)) | (SWIM_GOSSIP_USER_SPREAD << PER_BITS);
      slab.H(p) = hw;
    }
    // the next pass's hot bytes have arrived by now: its in-window gossips' receipt slots and the
    // first targets' receipt words are loaded here, so that the next pass's check hits the cache
    if (p + 64 < glen && (uint64_t)hn.inf_period() + spread >= period) {
      const uint32_t sn = gslot_of(gkey(hn.gossiper, hn.seq));
      sinkw ^= (uint32_t)gload(&c.gslot[sn].key);
      for (uint32_t jj = 0; jj < min(nt, 3u); ++jj) {
        const uint32_t tj = s_t[1 + jj];
        if (owned(c, tj)) sinkw ^= gload(&c.gbits[rbit_word(tj - c.lo, sn)]);
      }
    }
  }
  if (sinkw == 0x5bd1e995u && glen == 0x7fffffffu) set_err(c, 0u);  // keeps the warming loads; sets no bit
  PPROF_ACC(ep.t_pass, te1);
  // PAck waits on this member's LEAVING gossips (onLeavingDetected's spread() Monos): the gossips of
  // one wait share their infection period, so they complete together — in this round if it finds them
  // disseminated and the sweep has not dropped them (a swept gossip's Mono never completes)
  if (lane == 0 && sp.pw) {
    const uint32_t i = v - c.lo, np = min(c.pa_n[i], c.pa_cap);
    PAck* L = c.pa + (size_t)i * c.pa_cap;
    for (uint32_t k = 0; k < np; ++k) {
      const uint32_t gp = L[k].gp;
      if (gp && period > (uint64_t)(gp - 1) + spread && !(period > (uint64_t)(gp - 1) + sweep)) {
        L[k].gp = 0;
        L[k].ready = max(L[k].ready, (uint32_t)c.T);
      }
    }
  }
  const bool any_done = __ballot(done) != 0;
  if (lane == 0) {
    // the sweep dropped the prefix: the ring's base and the index's serial base advance past it
    GossipSched& gsv = gsched(c, v);
    gsv.base += lead;
    m.gix_base += lead;
    gsv.len = glen - lead;
    if (any_done) {
      m.leave_done = 1;
      c.mflag[v - c.lo] |= MF_LEAVE;
      if (c.xchg) {  // every shard stops sending to v at the end of this tick
        const uint32_t i = atomicAdd(&b.x->stop, 1u);
        if (i < b.tx_stop_cap) b.tx_stops[i] = v; else set_err(c, ERR_MSGS);
      }
    }
  }
  wave_order();
  return nmsg;
}

// doSpreadGossip's first steps for a due sender (one thread each, run by k_fd right after the
// member's FD step: both touch only the member's own state): period++ (:143) and, when it holds live
// gossips (:149-151), a place in the round's sender list (called by every lane of a wave: the list
// append is one atomic per wave)
__device__ __forceinline__ void gossip_round(const Ctx& c, const Bufs& b, uint32_t i) {
  bool busy = false;
  if (i < c.nl) {
    GossipSched gs = c.gs[i];  // one 16-B word per member
    const uint32_t t32 = (uint32_t)c.T;
    if (gs.next == t32) {  // the spreadGossip timer fires (phase g_start, period G; it runs while down too)
      gs.next = t32 + c.G;
      if (c.up[c.lo + i]) {
        gs.period++;  // period++ (:143); emit runs the round as period - 1
        // checkGossipSegmentation (:217-236): clear collectors holding more than the threshold of
        // intervals; only viewers whose collector crossed it since their last round look
        if (c.seg_flag[i]) {
          c.seg_flag[i] = 0;
          CollEnt* base = c.coll + (size_t)i * c.hcap;
          for (uint32_t j = 0; j < c.hcap; ++j)
            if (base[j].key && (int32_t)coll_size(c, base + j) > c.seg_threshold) {
              coll_clear(c, base + j);
              c.clr_tick[i] = (uint32_t)c.T;
              c.mem[i].clr_serial = c.mem[i].gix_base + gs.len;
            }
        }
        busy = gs.len != 0;  // else no target selection, no shuffle draw
      }
      c.gs[i].next = gs.next;
      c.gs[i].period = gs.period;
    }
  }
  const uint64_t mk = __ballot(busy);
  if (!mk) return;
  uint32_t base = 0;
  if ((threadIdx.x & 63) == 0) base = atomicAdd(&b.k->sender_cnt, (uint32_t)__popcll(mk));
  base = __shfl(base, 0, 64);
  if (busy) b.senders[base + lanes_below(mk)] = i;
}

// Phases A, B and C's first step.  256-thread workgroups, one viewer per thread.  The workgroup
// fires its viewers' due suspicion timers, compacts the ping / remote lists of its viewers that
// lost a member in the timer phase (a per-viewer dependency, so
// no separate launch), then every thread runs its viewer's FD step and, on gossip ticks, the
// first step of its gossip round (k_gossip_emit runs the rest after every FD step is done).
__device__ inline unsigned long long sync_collect_pre(const Ctx& c, const Bufs& b, uint32_t v, uint32_t sn, uint32_t fl);
__device__ inline unsigned long long sync_collect_member(const Ctx& c, const Bufs& b, uint32_t v);

// collect (ticks without a gossip round): the member's SYNC requests of phase D are collected here
// too, right after its FD step.  Nothing between k_fd and phase D on such a tick touches the state
// sync_collect_member reads (the member's own lists, schedule, fd_sync queue), so this equals the
// separate k_sync_collect launch and saves its round trips.
__global__ void __launch_bounds__(256) k_fd(KP, int gossip, int collect) {
  const Ctx c = pctx(P, T);
  __shared__ uint32_t s_list[256];
  __shared__ uint32_t s_cnt;
  if (c.xchg && blockIdx.x == 0 && threadIdx.x == 0) *P->b.rx_stop_n = 0;  // no leaves received yet
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // the member's schedule words, loaded alongside the timer queue's count (phase A changes none of
  // them; the FD step may set MF_FDSYNC, so mflag is reloaded after it)
  const uint32_t fdn = i < c.nl ? c.fd_next[i] : NONE;
  uint32_t sn = NONE, mfl = 0;
  if (collect && i < c.nl) {
    sn = c.sync_next[i];
    mfl = c.mflag[i];
  }
  timers_block(c, T);  // phase A for this block's viewers
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const bool flagged = i < c.nl && c.compact_flag[i] != 0;
  if (flagged) s_list[atomicAdd(&s_cnt, 1u)] = i;
  __syncthreads();
  const uint32_t nc = s_cnt;
  for (uint32_t k = 0; k < nc; ++k) {
    const uint32_t v = c.lo + s_list[k];
    MemberDev& m = mem(c, v);
    compact_list<256>(c, v, ping_list(c, v), m.ping_len);
    compact_list<256>(c, v, remote_list(c, v), m.remote_len);
  }
  if (flagged) c.compact_flag[i] = 0;
  __syncthreads();  // the compacted lengths are visible to every thread
  unsigned long long nev = 0, nreq = 0, npings = 0;
  if (i < c.nl && fdn == (uint32_t)T) {
    fd_member(c, c.lo + i, nev, nreq, npings);
    if (collect) mfl = c.mflag[i];
  }
  if (gossip) gossip_round(c, P->b, i);  // phase C's first step for this member
  if (collect) {
    const Ctx cs = pctx_sync(P, T);
    const unsigned long long nsync = i < c.nl ? sync_collect_pre(cs, P->b, c.lo + i, sn, mfl) : 0;
    wave_stat_add(cs, ST_SYNCS, nsync);
  }
  wave_stat_add(c, ST_FD_EVENTS, nev);
  wave_stat_add(c, ST_PING_REQS, nreq);
  wave_stat_add(c, ST_PINGS, npings);
}

// SWIM_DEBUG_SYNC: every exchange pointer a sharded tick dereferences (k_fd's rx_stop_n reset,
// k_recv_*, k_pack_rows, k_pull_rows, k_end_tick's counter reset and stop application, add_req's and
// emit's tx_* appends) is non-null when world > 1; an unsharded engine must never reach them (every
// use is guarded by world > 1 or by the owned() test, which is always true then)
__global__ void k_debug_exchange(KP) {
  const Ctx c = pctx(P, T);
  const Bufs& b = P->b;
  if (threadIdx.x != 0 || blockIdx.x != 0 || !c.xchg) return;
  const bool ok = b.x && b.tx_msgs && b.tx_reqs && b.tx_acks && b.tx_stops && b.tx_rows[0] && b.tx_rows[1] &&
                  b.peers && b.rx_cnt && b.rx_stops && b.rx_stop_n;
  if (!ok) atomicOr(c.err, ERR_XPTR);
}

// the rest of the round for the listed senders: one sender per wave at a time
// prof (sampled launches only): {GOSSIP_REQs materialised, live (gossip, sender) states, states whose
// hot bytes the round read: the swept prefix and the passes}
#ifndef EMIT_OCC
#define EMIT_OCC 4  // waves per SIMD the emit kernel is compiled for (its grid fills them: EMIT_GRID)
#endif
__global__ void __launch_bounds__(64 * EMIT_WAVES, EMIT_OCC) k_gossip_emit(KP, unsigned long long* prof) {
  __shared__ uint32_t s_t[EMIT_WAVES][98];
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t ns = b.k->sender_cnt;
  unsigned long long nmsg = 0, nmat = 0, nstate = 0, nexam = 0;
  EmitProf ep;
  // the wave's senders, up to 64 at a time: lane j loads the j-th one's index, schedule word and round
  // setup (SenderPre) in one batch of independent loads; then the senders run one after the other
  const uint32_t S = gridDim.x * EMIT_WAVES;
  for (uint32_t k0 = __builtin_amdgcn_readfirstlane(blockIdx.x * EMIT_WAVES + wv); k0 < ns; k0 += 64 * S) {
    const uint32_t kj = k0 + lane * S;
    uint32_t pi = 0, plen = 0, pper = 0, pbase = 0;
    SenderPre pre;
    pre.ok = 0;
    pre.rlen = 0;
    pre.idx = -1;
    pre.fut = 0;
    if (kj < ns) {
      pi = b.senders[kj];
      const GossipSched g = c.gs[pi];
      plen = g.len;
      pper = g.period;
      pbase = g.base;
      sender_pre_load(c, b, pi, pre);
    }
    const uint32_t nb = min(64u, (ns - k0 + S - 1) / S);
    // the two ends of a sender's slab (its first and last 64 states), loaded one sender ahead
    auto slab_ends = [&](uint32_t j, GossipHot& hh, GossipHot& ht) {
      const uint32_t i = rdlane(pi, j), glen = rdlane(plen, j), gb = rdlane(pbase, j);
      const SlabRef sl = slab_of(c, c.lo + i, gb);
      hh = GossipHot{};
      ht = GossipHot{};
      if (lane < glen) hh = sl.Hg(lane);
      if (glen > 64 && glen - 64 + lane < glen) ht = sl.Hg(glen - 64 + lane);
    };
    GossipHot ch, ct;
    if (nb) slab_ends(0, ch, ct);
    for (uint32_t j = 0; j < nb; ++j) {
      const uint32_t i = rdlane(pi, j);
      const uint32_t glen = rdlane(plen, j);
      const uint32_t per = rdlane(pper, j);
      const uint32_t gb = rdlane(pbase, j);
      const SenderPre sp = sender_pre_from(pre, (int)j);
      GossipHot nh{}, nt{};
      if (j + 1 < nb) slab_ends(j + 1, nh, nt);
      nstate += glen;
      nmsg += gossip_emit_sender(c, b, c.lo + i, per - 1, glen, gb, lane, s_t[wv], nmat, nexam, ep, sp, ch, ct);
      ch = nh;
      ct = nt;
    }
  }
  PPROF_CNT(16, ep.t_setup);
  PPROF_CNT(17, ep.t_pass);
  PPROF_CNT(18, ep.t_win);
  PPROF_CNT(19, ep.t_mat);
  PPROF_CNT(20, ep.n_all);
  PPROF_CNT(21, ep.n_win);
  PPROF_CNT(22, ep.n_mat);
  PPROF_CNT(23, ep.n_snd);
  PPROF_CNT(24, ep.t_sel);
  PPROF_CNT(25, ep.t_tgt);
  if (lane == 0 && nmat) atomicAdd(&b.k->msg_total, (uint32_t)nmat);
  if (prof && lane == 0 && nstate) {
    atomicAdd(prof, nmat);
    atomicAdd(prof + 1, nstate);
    atomicAdd(prof + 2, nexam);
  }
  wave_stat_add(c, ST_GOSSIP_MESSAGES, nmsg);
}

// GOSSIP_REQs delayed by the network emulator that arrive in tick T join the inboxes (one launch of
// ceil(cnt / 256) workgroups; emit never writes the bucket of the current tick, and k_end_tick empties
// it).  Each (receiver, sending tick, sender) group gets pseq dense in slab-position order, as emit
// gives a round's fresh messages, so the deliverer ranks them by their snd_key.
__global__ void __launch_bounds__(256) k_dq_release(KP) {
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  const uint32_t bk = (uint32_t)T & DQ_MASK;
  const uint32_t cnt = min(b.dq_cnt[bk], b.dq_bcap);
  const GMsgFull* q = b.dq + (size_t)bk * b.dq_bcap;
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i0 = blockIdx.x * blockDim.x + (threadIdx.x - lane); i0 < cnt; i0 += gridDim.x * blockDim.x) {
    const uint32_t i = i0 + lane;
    bool valid = i < cnt;
    GMsgFull msg{};
    uint32_t age = 0;
    if (valid) {
      msg = q[i];
      // the receiver's inbound filter when the message arrives (listen() :78-83); it depends on the
      // (receiver, sender) pair only, so a dropped pair's ranks vanish together and the others stay dense
      valid = in_pass(c, msg.to, msg.from);
    }
    if (valid) {
      uint32_t rank = 0;
      for (uint32_t j = 0; j < cnt; ++j) {
        const GMsgFull& o = q[j];
        // copies with equal keys (one gossip sent to two targets at one address) are identical
        // messages: ranked in bucket order
        rank += (o.to == msg.to && o.pseq == msg.pseq && o.from == msg.from &&
                 (o.pos() < msg.pos() || (o.pos() == msg.pos() && j < i))) ? 1u : 0u;
      }
      age = (uint32_t)T - msg.pseq;  // snd_key orders earlier rounds first
      msg.pseq = rank;
      if (!owned(c, msg.to)) {
        // a receiver on another shard: the message joins this tick's exchange (E1), its age in the
        // top bits of `from` (< 2^20 while delays are on; k_recv_msgs takes it out)
        GMsgFull fm = msg;
        fm.from |= min(age, 2047u) << 20;
        const uint32_t d = owner(c, msg.to);
        const uint32_t bj = atomicAdd(&b.x->msg[d], 1u);
        if (bj < b.tx_msg_cap) b.tx_msgs[(size_t)d * b.tx_msg_cap + bj] = fm; else set_err(c, ERR_MSGS);
        valid = false;
      }
    }
    deliver_local_msg(c, b, msg, valid, age);  // every lane of the wave takes part
  }
}

// ------------------------------------------------------------------------------- exchange
// A system-scope load: coherent with another GPU's finished stores (exchange buffers over xGMI; in a
// local group it is an ordinary load of this device's memory that bypasses nothing it needs).
template <typename T>
__device__ __forceinline__ T ld_peer(const T* p) {
  static_assert(sizeof(T) % 8 == 0, "8-byte granules");
  T v;
  const uint64_t* s = reinterpret_cast<const uint64_t*>(p);
  uint64_t* d = reinterpret_cast<uint64_t*>(&v);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 8); ++i) d[i] = __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return v;
}
__device__ __forceinline__ uint32_t ld_peer_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// What each peer produced for this shard this tick, clamped to the exchange capacity, loaded by the
// workgroup into LDS (a register array indexed by peer would live in scratch); returns the total.
__device__ __forceinline__ uint32_t peer_counts(const Ctx& c, const Bufs& b, uint32_t kind, uint32_t cap, uint32_t* s_n) {
  if (threadIdx.x < (uint32_t)MAXW) {
    const uint32_t p = threadIdx.x;
    s_n[p] = p < c.world && p != c.rank ? min(b.rx_cnt[kind * MAXW + p], cap) : 0u;
  }
  __syncthreads();
  uint32_t total = 0;
  for (uint32_t p = 0; p < (uint32_t)MAXW; ++p) total += s_n[p];
  return total;
}
// flat index i < total -> (peer, index among that peer's items)
__device__ __forceinline__ uint32_t peer_of(const uint32_t* s_n, uint32_t& i) {
  uint32_t p = 0;
  while (i >= s_n[p]) { i -= s_n[p]; ++p; }
  return p;
}

// Local group only: the counts each peer shard produced for this one (what ncclAllToAll /
// ncclAllGather deliver to a rank), read from the peers' counters.
__global__ void k_gather_counts(KP, int kind) {
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  const uint32_t p = threadIdx.x;
  if (p >= (uint32_t)MAXW) return;
  uint32_t n = 0, stop = 0;
  if (p < c.world && p != c.rank) {
    const Xc& x = *b.peers->x[p];
    n = kind == XK_MSG ? x.msg[c.rank] : kind == XK_REQ ? x.req[c.rank] : x.ack[c.rank];
    stop = x.stop;
  }
  b.rx_cnt[kind * MAXW + p] = n;
  if (kind == XK_MSG) b.rx_cnt[XK_STOP * MAXW + p] = stop;
}

// E1: GOSSIP_REQs other shards produced for receivers owned here join the inboxes exactly as a local
// send does (read straight from the producers' tx buffers); provable duplicates (the emitter could
// not see this shard's collectors) are flagged, and delivery skips them: the collector holds the
// sequence id, so onGossipReq would return at once.  Workgroup 0 also takes the peers' completed
// graceful leaves (k_end_tick applies them).  The work size is read on the device: a fixed grid.
__global__ void k_recv_msgs(KP) {
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  const Peers* pr = b.peers;
  __shared__ uint32_t s_n[MAXW], s_st[MAXW];
  if (blockIdx.x == 0) {
    peer_counts(c, b, XK_STOP, b.tx_stop_cap, s_st);
    uint32_t o = 0;
    for (uint32_t p = 0; p < c.world; ++p) {
      for (uint32_t j = threadIdx.x; j < s_st[p]; j += blockDim.x) b.rx_stops[o + j] = ld_peer_u32(pr->stops[p] + j);
      o += s_st[p];
    }
    if (threadIdx.x == 0) *b.rx_stop_n = o;
  }
  const uint32_t total = peer_counts(c, b, XK_MSG, b.tx_msg_cap, s_n);
  // wave-uniform trip count: every lane of a wave takes part in each deliver_local_msg call
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i0 = blockIdx.x * blockDim.x + (threadIdx.x - lane); i0 < total; i0 += gridDim.x * blockDim.x) {
    uint32_t i = i0 + lane;
    const bool valid = i < total;
    GMsgFull msg{};
    uint32_t age = 0;
    if (valid) {
      const uint32_t p = peer_of(s_n, i);
      msg = ld_peer(pr->msgs[p] + (size_t)c.rank * b.tx_msg_cap + i);
      if (c.delay_on) {  // a delayed message released by its sender's shard (k_dq_release)
        age = msg.from >> 20;
        msg.from &= 0xfffffu;
      }
      // kept (flagged) so that each (sender, receiver) pair's pseq stays dense for deliver_big
      if (coll_contains(c, coll_find(c, msg.to, msg.gossiper), msg.seq)) msg.pos_dup |= 0x80000000u;
    }
    deliver_local_msg(c, b, msg, valid, age);
  }
}

// inboxes above DLV_SORT messages are delivered by a whole wave (deliver_big)
#ifndef DLV_SORT_N
#define DLV_SORT_N 24
#endif
constexpr int DLV_SORT = DLV_SORT_N;

// canonical sender key: earlier sending rounds first (a released delayed message's pad holds its age
// in ticks, DQ: n <= 2^20 when delays are on), then the sender
__device__ __forceinline__ uint32_t snd_key(const Ctx& c, const GMsgFull& g) {
  return c.delay_on ? ((4095u - min(g.to, 4095u)) << 20) | g.from : g.from;
}
__device__ __forceinline__ uint64_t msg_key(const Ctx& c, const GMsgFull& m) {
  return ((uint64_t)snd_key(c, m) << 32) | m.pos();
}


// The next message's lines, loaded while the current one is processed: its collector slot, its
// receipt-bitmap slot, the view cell and reference record of its subject — the dependent loads its
// onGossipReq starts with, so that they hit the cache (values are re-read, never trusted: the current
// message may change them).  Returns a value the caller folds into a sink that is never true.
__device__ __forceinline__ uint32_t warm_gossip_req(const Ctx& c, uint32_t r, const CollEnt* cbase, const GMsgFull& g) {
#ifdef SWIM_DLV_NO_WARM  // (profiling A/B builds only)
  return 0;
#endif
  uint32_t x = cbase[hash32(g.gossiper) & (c.hcap - 1)].key;
  const uint32_t sl = gslot_of(gkey(g.gossiper, g.seq));
  x ^= (uint32_t)c.gslot[sl].key ^ (uint32_t)c.gpend[sl];
  if (g.status() < SWIM_GOSSIP_USER && g.subject < c.n) {
    const size_t i = (size_t)(r - c.lo) * c.n + g.subject;
    x ^= c.recs[i] ^ c.aux[i] ^ c.ref[g.subject];
  }
  return x;
}

// onGossipReq (GossipProtocolImpl.java:201-215) for one received message, in canonical order
// onGossipReq after the collector accepted the sequence id (and the receipt bit is marked): the
// gossip's state is appended and onMembershipGossip runs, or — only if `lookup` (the collector was
// cleared, and states older than the clear are still in the slab) — a state that outlived the clear
// takes the sender as infected
__device__ __forceinline__ void gossip_accepted(const Ctx& c, uint32_t r, MemberDev& m, const SlabRef& slab, const GMsgFull& g,
                                       bool lookup) {
  PPROF_T0(tc);
  const int32_t found = lookup ? gix_find(c, m, r, slab, g.gossiper, g.seq) : -1;
  if (found < 0) {
    GossipSched& gs = gsched(c, r);
    if (gs.len >= c.gcap) { set_err(c, ERR_SLAB); return; }
    GossipDev ns;
    ns.gossiper = g.gossiper; ns.seq = g.seq; ns.subject = g.subject; ns.status = g.status(); ns.inc = g.inc();
    ns.inf_period = gs.period;
    ns.inf[0] = g.from;
#pragma unroll
    for (int k = 1; k < GINF; ++k) ns.inf[k] = NONE;
    if (gs.period > PER_MASK) set_err(c, ERR_INC);  // (2^28 gossip rounds)
    slab.put(gs.len++, ns);
    gix_note(c, m, r, ns.gossiper, ns.seq);
    PPROF_WADD(8, tc);
    PPROF_T0(td);
    if (g.status() >= SWIM_GOSSIP_USER)  // sink.next(gossip.message()) (:209): listen() subscribers
      emit(c, r, g.gossiper, SWIM_EV_GOSSIP, SWIM_PHASE_GOSSIP, m.ev_minor++, g.subject);
    // onMembershipGossip (MembershipProtocolImpl.java:452-459)
    else if (update_membership(c, r, g.subject, g.status(), g.inc(), R_GOSSIP, SWIM_PHASE_GOSSIP))
      apply_alive(c, r, g.subject, g.inc(), R_GOSSIP, SWIM_PHASE_GOSSIP);
    PPROF_WADD(9, td);
  } else {
    GossipDev st = slab.get((uint32_t)found);
    if (!gossip_infected(st, g.from)) {
      // the first free slot, written through an unrolled select: a runtime index would put the
      // whole array in scratch
      bool put = false;
#pragma unroll
      for (int k = 0; k < GINF; ++k) {
        const bool here = !put && st.inf[k] == NONE;
        st.inf[k] = here ? g.from : st.inf[k];
        put |= here;
      }
      if (put) slab.put((uint32_t)found, st);
      else set_err(c, ERR_INFECTED);
    }
  }
}
__device__ inline bool on_gossip_req(const Ctx& c, uint32_t r, MemberDev& m, const SlabRef& slab, const GMsgFull& g) {
  if (g.dup()) return false;  // the collector held it on arrival and only grows until now
  CollEnt cv;
  CollEnt* col = coll_ensure_v(c, r, g.gossiper, cv);
  if (!col) return false;
  const bool was_cleared = (cv.meta & COLL_CLEARED) != 0;
  const bool added = coll_add(c, col, g.seq, &c.seg_flag[r - c.lo], &cv);
  if (!added) return false;
  receipt_mark(c, r, g.gossiper, g.seq);
  // a GossipState can outlive its collector entry only after a clear
  gossip_accepted(c, r, m, slab, g, was_cleared && pre_clear_states(m));
  return true;
}

// ------------------------------------------------------------------------------- list inserts
// group barrier of apply_ins_batch: the workgroup, or one wave (global and LDS accesses of the wave
// complete before any lane goes on)
template <bool WG>
__device__ __forceinline__ void ins_bar() {
  if (WG) {
    __syncthreads();
  } else {
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
  }
}

// pingMembers.add(nextInt(size), s) (FailureDetectorImpl.java:334-345) for every ADDED event of
// viewer v in this phase, in event order, in ONE pass over the list: the inserts' final positions are
// resolved first (insert q shifts every earlier insert at or after its index), then the original
// elements move right, tail first, by the number of inserted positions before their destination, then
// the inserted members are written — the list k sequential ArrayList.add calls leave.  NT threads
// cooperate (a workgroup, WG = true, or one wave); every thread of the group calls it.  sP / sS / sR:
// NT words of LDS each.
#ifndef INS_U
#define INS_U 4  // list elements a thread moves per step of apply_ins_batch (1: one, for A/B)
#endif
template <int NT, bool WG>
__device__ __forceinline__ void apply_ins_batch(const Ctx& c, uint32_t v, uint32_t tid, uint32_t* sP, uint32_t* sS, uint32_t* sR) {
  MemberDev& m = mem(c, v);
  const uint32_t k = m.ins_rank;
  if (k == 0) return;
  uint32_t* pl = ping_list(c, v);
  const InsOp* inl = c.ins_inline + (size_t)(v - c.lo) * INS_INLINE;
  uint32_t blk = m.ins_head, blk_idx = 0;  // (thread 0: the block its hops have reached)
  uint32_t len = m.ping_len;
  for (uint32_t q0 = 0; q0 < k; q0 += NT) {
    const uint32_t kb = min((uint32_t)NT, k - q0);
    // index of insert q = nextInt(size before it); the draw is keyed by the event (phase, minor)
    if (tid < kb && q0 + tid < INS_INLINE) {
      const InsOp op = inl[q0 + tid];
      sS[tid] = op.s;
      sP[tid] = next_int(draw(c, v, SWIM_STREAM_PING_INSERT, op.phase, op.minor), len + tid);
    }
    if (q0 + kb > INS_INLINE) {  // the batch's ops in blocks: their starts into sR (thread 0), then the ops
      uint32_t o, z;
      const uint32_t b0 = ins_block_of(q0 > INS_INLINE ? q0 - INS_INLINE : 0u, o, z);
      const uint32_t b1 = ins_block_of(q0 + kb - 1 - INS_INLINE, o, z);
      if (tid == 0) {
        for (; blk_idx < b0; ++blk_idx) blk = c.ins[blk].next;
        sR[0] = blk;
        for (uint32_t bb = b0 + 1; bb <= b1; ++bb) {
          blk = c.ins[blk].next;
          sR[bb - b0] = blk;
        }
        blk_idx = b1;
      }
      ins_bar<WG>();
      if (tid < kb && q0 + tid >= INS_INLINE) {
        const uint32_t bq = ins_block_of(q0 + tid - INS_INLINE, o, z);
        const InsOp op = c.ins[sR[bq - b0] + o];
        sS[tid] = op.s;
        sP[tid] = next_int(draw(c, v, SWIM_STREAM_PING_INSERT, op.phase, op.minor), len + tid);
      }
    }
    ins_bar<WG>();
    for (uint32_t q = 1; q < kb; ++q) {  // sP[j] -> position of insert j after insert q
      const uint32_t idx = sP[q];
      if (tid < q && sP[tid] >= idx) sP[tid] += 1;
      ins_bar<WG>();
    }
    if (tid < kb) {  // final positions ascending (they are distinct)
      const uint32_t p = sP[tid];
      uint32_t rk = 0;
      for (uint32_t j = 0; j < kb; ++j) rk += sP[j] < p ? 1u : 0u;
      sR[rk] = p;
    }
    ins_bar<WG>();
    // original element i lands at i + #{j : sR[j] - j <= i} (sR[j] - j is non-decreasing).  The
    // elements move tail first, INS_U * NT per step: the step's loads, one group barrier, its stores.
    // A step stores at or above its lowest source and the next step loads below it, so only a step's
    // own loads must precede its stores (one barrier a step, where one element a thread took two).
    const uint32_t pmin = sR[0];
    for (int64_t hi = (int64_t)len; hi > (int64_t)pmin; hi -= (int64_t)NT * INS_U) {
      uint32_t val[INS_U], dest[INS_U];
#pragma unroll
      for (int u = 0; u < INS_U; ++u) {
        const int64_t i = hi - (int64_t)NT * (u + 1) + tid;
        val[u] = 0;
        dest[u] = NONE;
        if (i >= (int64_t)pmin) {
          val[u] = pl[i];
          uint32_t a = 0, z = kb;
          while (a < z) {
            const uint32_t mid = (a + z) >> 1;
            if (sR[mid] - mid <= (uint32_t)i) a = mid + 1; else z = mid;
          }
          dest[u] = (uint32_t)i + a;
        }
      }
      ins_bar<WG>();
#pragma unroll
      for (int u = 0; u < INS_U; ++u)
        if (dest[u] != NONE) pl[dest[u]] = val[u];
    }
    // (the inserted members' slots are no move's destination, and every move's load was waited on)
    if (tid < kb) pl[sP[tid]] = sS[tid];
    len += kb;
    ins_bar<WG>();
  }
  if (tid == 0) {
    m.ping_len = len;
    m.ins_rank = 0;
  }
  ins_bar<WG>();
}

// ------------------------------------------------------------------------------- delivery
// Small inboxes (<= DLV_SORT messages): one receiver per thread, the inbox keys (sender, slab
// position) insertion-sorted in an LDS slice laid out [slot][thread] (conflict-free), then
// onGossipReq in that order.  Big inboxes: one wave per receiver (deliver_big).
constexpr int DLV_BLOCK = 256;
constexpr int DLV_WAVES = DLV_BLOCK / 64;
constexpr uint32_t BIG_MAXD = 128;  // distinct senders a big inbox is ranked over in LDS

// (nfresh: messages not flagged as provable duplicates, i.e. that ran the collector check)
__device__ inline unsigned long long deliver_sorted(const Ctx& c, uint32_t r, const GMsgFull* a, uint32_t k,
                                                    const uint8_t* ix8, uint32_t ix8_stride, uint32_t& nfresh) {
  MemberDev& m = mem(c, r);
  m.ev_minor = 0;
  m.fetch_ctr = 0;
  const SlabRef slab = slab_of(c, r);
  const CollEnt* cbase = c.coll + (size_t)(r - c.lo) * c.hcap;
  unsigned long long acc = 0;
  uint32_t sink = 0;
  GMsgFull next = a[ix8 ? ix8[0] : 0];
  for (uint32_t q = 0; q < k; ++q) {
    const GMsgFull g = next;
    if (q + 1 < k) {
      next = a[ix8 ? ix8[(q + 1) * ix8_stride] : q + 1];
      sink ^= warm_gossip_req(c, r, cbase, next);
    }
    nfresh += g.dup() ? 0u : 1u;
    if (on_gossip_req(c, r, m, slab, g)) acc++;
  }
  if (sink == 0x5bd1e995u && k == 0x7fffffffu) set_err(c, 0u);  // keeps the warming loads; sets no bit
  return acc;
}

struct BigLds {  // per wave
  uint32_t snd[BIG_MAXD];  // distinct senders (found order, then ascending)
  uint32_t cnt[BIG_MAXD];  // their message counts, then running inbox bases
  uint32_t iP[64], iS[64], iR[64];  // apply_ins_batch scratch
  uint32_t perm[64];  // an inbox of at most 64 messages ranked for the whole-wave delivery: rank -> slot
};

__device__ __forceinline__ void wave_sync() {
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}

// slot of sender sf among the nd listed (wave-uniform result), or -1
__device__ __forceinline__ int big_find(const uint32_t* snd, uint32_t nd, uint32_t sf, uint32_t lane) {
  for (uint32_t j0 = 0; j0 < nd; j0 += 64) {
    const uint32_t j = j0 + lane;
    const uint64_t hit = __ballot(j < nd && snd[j] == sf);
    if (hit) return (int)(j0 + (uint32_t)__ffsll((unsigned long long)hit) - 1);
  }
  return -1;
}

// Big inboxes, up to 64 per wave.  Canonical order is (sender, slab position), and it needs no
// comparison sort: k_gossip_emit numbers each (sender, receiver) pair's messages of the round in
// slab-position order (GMsgFull.pseq, dense: every materialised message reaches the inbox, cross-
// shard duplicates included, flagged), so rank = base of the sender (senders ascending by snd_key,
// bases from their message counts) + pseq.  The wave ranks its receivers one after the other (all
// lanes on one inbox), then lane j runs receiver j's onGossipReq chain in rank order — the chains
// of the batch run side by side, each touching only its own receiver's state — then, receiver by
// receiver, the inbox pages go back, the pingMembers inserts of the phase run and the SYNC
// collection follows.
// lds_perm: an inbox of at most 64 messages keeps its permutation in L.perm instead of pg_perm (the
// whole-wave delivery reads it from there: no dependent global round trip before its messages).
__device__ __forceinline__ uint32_t rank_big_inbox(const Ctx& c, const Bufs& b, uint32_t i, uint32_t k, uint32_t lane, BigLds& L,
                                   bool lds_perm = false) {
  const uint32_t* pt = b.pg_tab + (size_t)i * b.pg_max;
  auto msg_at = [&](uint32_t q) -> const GMsgFull& { return b.pg_msgs[(size_t)pt[q >> 6] * 64 + (q & 63)]; };
  auto perm_at = [&](uint32_t q) -> uint32_t& { return b.pg_perm[(size_t)pt[q >> 6] * 64 + (q & 63)]; };
  // pass 1: distinct senders and their message counts
  uint32_t nd = 0;
  bool over = false;
  for (uint32_t q0 = 0; q0 < k && !over; q0 += 64) {
    const uint32_t q = q0 + lane;
    const uint32_t f = q < k ? snd_key(c, msg_at(q)) : NONE;
    uint64_t todo = __ballot(q < k);
    while (todo) {
      const uint32_t sf = rdlane(f, (uint32_t)__ffsll((unsigned long long)todo) - 1);
      const uint64_t same = __ballot(f == sf) & todo;
      int slot = big_find(L.snd, nd, sf, lane);
      if (slot < 0) {
        if (nd == BIG_MAXD) { over = true; break; }
        slot = (int)nd;
        if (lane == 0) { L.snd[nd] = sf; L.cnt[nd] = 0; }
        nd++;
      }
      if (lane == 0) L.cnt[slot] += (uint32_t)__popcll(same);
      wave_sync();
      todo &= ~same;
    }
  }
  if (over) {
    // more distinct senders than the LDS table holds (needs > BIG_MAXD senders choosing this
    // receiver in one round): senders one at a time, ascending, by repeated minimum search
    uint32_t lo_s = 0, rank = 0;
    for (;;) {
      uint32_t mn = NONE;
      for (uint32_t q = lane; q < k; q += 64) {
        const uint32_t f = snd_key(c, msg_at(q));
        if (f >= lo_s && f < mn) mn = f;
      }
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) mn = min(mn, (uint32_t)__shfl_xor(mn, d, 64));
      if (mn == NONE) break;
      uint32_t cnt = 0;
      for (uint32_t q0 = 0; q0 < k; q0 += 64) {
        const uint32_t q = q0 + lane;
        const bool mine = q < k && snd_key(c, msg_at(q)) == mn;
        if (mine && rank + msg_at(q).pseq < k) perm_at(rank + msg_at(q).pseq) = q;
        cnt += (uint32_t)__popcll(__ballot(mine));
      }
      rank += cnt;
      lo_s = mn + 1;
    }
  } else {
    // senders ascending, inbox bases = exclusive prefix of their counts in that order
    uint32_t ms[2], mc[2], mr[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t j = lane + 64u * t;
      ms[t] = j < nd ? L.snd[j] : NONE;
      mc[t] = j < nd ? L.cnt[j] : 0u;
      mr[t] = 0;
      if (j < nd)
        for (uint32_t x = 0; x < nd; ++x) mr[t] += L.snd[x] < ms[t] ? 1u : 0u;
    }
    wave_sync();
#pragma unroll
    for (int t = 0; t < 2; ++t)
      if (lane + 64u * t < nd) { L.snd[mr[t]] = ms[t]; L.cnt[mr[t]] = mc[t]; }
    wave_sync();
    if (lane == 0) {
      uint32_t acc0 = 0;
      for (uint32_t x = 0; x < nd; ++x) { const uint32_t t = L.cnt[x]; L.cnt[x] = acc0; acc0 += t; }
    }
    lds_perm = lds_perm && k <= 64u;
    if (lds_perm) L.perm[lane] = NONE;  // (a rank left unwritten is a hole, as in pg_perm)
    wave_sync();
    // pass 2: rank = base of the sender + the message's pseq (dense per (sender, receiver))
    for (uint32_t q0 = 0; q0 < k; q0 += 64) {
      const uint32_t q = q0 + lane;
      uint32_t f = NONE, ps = 0;
      if (q < k) {
        const GMsgFull& g = msg_at(q);
        f = snd_key(c, g);
        ps = g.pseq;
      }
      uint64_t todo = __ballot(q < k);
      while (todo) {
        const uint32_t sf = rdlane(f, (uint32_t)__ffsll((unsigned long long)todo) - 1);
        const uint64_t same = __ballot(f == sf) & todo;
        const uint32_t at = L.cnt[big_find(L.snd, nd, sf, lane)] + ps;
        if (((same >> lane) & 1ull) && at < k) {
          if (lds_perm) L.perm[at] = q;
          else perm_at(at) = q;
        }
        todo &= ~same;
      }
    }
  }
  wave_sync();
  return k;
}

// Whole-wave delivery of one big inbox (k >= b.coop_min ranked messages): the same onGossipReq
// sequence (GossipProtocolImpl.java:201-215) as the lane chain, 64 ranks at a time.
//  (a) collectors: each gossiper of the chunk gets one leader lane, which adds its lanes' sequence ids
//      in rank order (a collector's intervals — and the segmentation flag — see the same sequence of
//      adds as in the chain); leaders of different gossipers run side by side (two finding one empty
//      table slot are told apart by ballot, coll_ensure_wave: no compare-and-swap round trip).  A lane whose add fails holds a copy the collector already had:
//      rejected, as in the chain.  Messages of the member's own gossips take the chain's own
//      onGossipReq at their turn in (c) instead.  A collector that was cleared takes its adds here as
//      well; while states older than the clear are still in the slab (pre_clear_states) its accepted
//      lanes look their state up at their turn in (c) (a GossipState may outlive the clear: gix_find,
//      the index rebuilt by the whole wave when needed), which takes one serial step each instead of
//      a single-lane collector add over thousands of intervals.
//  (b) receipt marks of the accepted lanes; then which accepted records cannot change the view: the
//      namespace filter drops them, or they do not override the subject's record as it stands after
//      the earlier chunks and no earlier lane of the chunk may change that subject
//      (MembershipRecord.isOverrides, updateMembership :593-602) — their onMembershipGossip is a no-op.
//  (c) in rank order, lane by lane, the others: slab position and state, then onMembershipGossip (or
//      the user gossip's listen() event) — which may spread gossips (slab appends) and emit events;
//      the no-op lanes between them take the next positions and write their states together.
// Returns this lane's share of the accepted messages; nfresh counts those not flagged as provable
// duplicates (per lane as well).
// lane i gets lane i + 1's / i - 1's value (DPP wave_shl:1 / wave_shr:1, GFX9: one VALU op across the
// whole wave, no LDS crossbar round trip); the lane at the end keeps its own
__device__ __forceinline__ uint32_t wave_from_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_from_prev(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xf, 0xf, false);
}
#ifndef COOP_STAGE
#define COOP_STAGE 1  // spilled collectors' adds staged in LDS (0: coll_add one by one, for A/B)
#endif
#ifndef COOP_PIPE
#define COOP_PIPE 1  // the chunk pipeline below (0: the next chunk's loads waited on at its start)
#endif
constexpr uint32_t COOP_LIV = 2048;  // intervals of one collector staged in LDS per wave (16 KB)
constexpr uint32_t COOP_MIN = 16;  // Bufs.coop_min's default (every big inbox: measured best, 16 / 32 / 64)
// gix_find's rebuild of the slab index made by a whole wave (the first lookup a cleared collector
// needs in the whole-wave delivery): the table emptied 64 slots at a time, the slab's len states
// inserted 64 at a time (gix_put_atomic), where one lane takes mask + 1 stores and len dependent
// inserts (2^19 and ~10^5 at config 3's churn)
__device__ inline void gix_rebuild_wave(const Ctx& c, MemberDev& m, uint32_t v, const SlabRef& slab, uint32_t len,
                                        uint32_t lane) {
  uint32_t* ix = gix_of(c, v);
  const uint32_t mask = c.gix_mask;
  const uint32_t base = __builtin_amdgcn_readfirstlane(m.gix_base);
  for (uint32_t q = lane; q <= mask; q += 64) ix[q] = NONE;
  wave_sync();
  uint32_t took = 0;
  for (uint32_t p0 = 0; p0 < len; p0 += 64) {
    const uint32_t p = p0 + lane;
    if (p < len) {
      const GossipHot h = slab.Hg(p);
      took += gix_put_atomic(ix, mask, base, len, h.gossiper, h.seq, base + p) ? 1u : 0u;
    }
  }
  took = (uint32_t)wave_sum(took);
  if (lane == 0) {
    m.gix_used = took;
    m.gix_valid = 1;
  }
  wave_sync();
}

__device__ __forceinline__ unsigned long long deliver_coop(const Ctx& c, const Bufs& b, uint32_t i, uint32_t k, uint32_t lane, BigLds& L,
                                           uint2* siv, uint32_t& nfresh) {
  const uint32_t r = c.lo + i;
  const uint32_t* pt = b.pg_tab + (size_t)i * b.pg_max;
  MemberDev& m = mem(c, r);
  GossipSched& gsr = gsched(c, r);
  const SlabRef slab = slab_of(c, r);
  if (lane == 0) {
    m.ev_minor = 0;
    m.fetch_ctr = 0;
  }
  uint32_t len = __builtin_amdgcn_readfirstlane(gsr.len);
  const uint32_t period = gsr.period;
  // no state predates the last collector clear: a cleared collector's adds are made in (a) like any
  // other's, and the slab index need not be kept up (pre_clear_states)
  const bool pre = pre_clear_states(m);
  if (!pre && lane == 0 && m.gix_valid) m.gix_valid = 0;
  if (lane == 0 && period > PER_MASK) set_err(c, ERR_INC);  // (2^28 gossip rounds)
  unsigned long long acc = 0;
  // The messages in rank order, pipelined across chunks: a chunk's messages are loaded at the start
  // of the chunk before it, their slots (pg_perm) one chunk earlier still, and the first 64 page ids
  // are held one per lane — so a chunk waits on no dependent load of its own.  An inbox of one page
  // has its permutation in LDS (rank_big_inbox).
  const bool one_page = k <= 64u;
  const uint32_t npg = (k + 63) / 64;
  const uint32_t ptl = lane < npg ? gload(pt + lane) : 0u;
  const uint32_t pg0 = rdlane(ptl, 0);
  auto slot_of = [&](uint32_t q) -> uint32_t {  // rank q's slot; (q >> 6) is the same on every lane
    if (one_page) return q < k ? L.perm[q] : NONE;
    const uint32_t pgi = __builtin_amdgcn_readfirstlane(q >> 6);
    const uint32_t pg = pgi < 64u ? rdlane(ptl, pgi) : __builtin_amdgcn_readfirstlane(gload(pt + pgi));
    return q < k ? gload(b.pg_perm + (size_t)pg * 64 + (q & 63)) : NONE;
  };
  auto msg_at = [&](uint32_t q, uint32_t jq) -> GMsgFull {  // (every lane calls it: the page shuffle)
    const bool ok = q < k;
    if (ok && jq >= k) {  // a hole: only after an inbox overflow (ERR_MSGS is set)
      set_err(c, ERR_MSGS);
      jq = q;
    }
    const uint32_t pgi = ok ? jq >> 6 : 0u;
    const uint32_t viaL = (uint32_t)__shfl((int)ptl, (int)(pgi & 63u), 64);
    GMsgFull x{};
    if (ok) x = b.pg_msgs[(size_t)(one_page ? pg0 : pgi < 64u ? viaL : gload(pt + pgi)) * 64 + (jq & 63)];
    return x;
  };
  const CollEnt* cbase = c.coll + (size_t)i * c.hcap;
  uint32_t sink = 0;
  GMsgFull gn = msg_at(lane, slot_of(lane));
#if COOP_PIPE
  uint32_t jn = k > 64u ? slot_of(64u + lane) : NONE;  // the next chunk's slots
#endif
  wave_sync();
  for (uint32_t r0 = 0; r0 < k; r0 += 64) {
    PPROF_T0(tca);
    const uint32_t q = r0 + lane;
    const GMsgFull g = gn;
    const bool valid = q < k && !g.dup();
    nfresh += valid ? 1u : 0u;
    const bool more = r0 + 64 < k;
    if (more) {
#if COOP_PIPE
      gn = msg_at(q + 64, jn);
      jn = r0 + 128 < k ? slot_of(q + 128) : NONE;
#else
      gn = msg_at(q + 64, slot_of(q + 64));
      if (q + 64 < k) sink ^= cbase[hash32(gn.gossiper) & (c.hcap - 1)].key;
#endif
    }
    // (a) one leader per gossiper
    const bool coop = valid && g.gossiper != r;
    L.iP[lane] = g.seq;
    L.iS[lane] = 0;  // 1: accepted, 2: onGossipReq at its turn
    uint64_t grp = 0;
    const uint64_t coopm = __ballot(coop);
    PPROF_ADD(29, tca);
    PPROF_T0(tcg);
    for (uint64_t todo = coopm; todo;) {
      const int l = __ffsll((unsigned long long)todo) - 1;
      const uint32_t gl = rdlane(g.gossiper, (uint32_t)l);
      const uint64_t same = __ballot(coop && g.gossiper == gl) & todo;
      if (lane == (uint32_t)l) grp = same;
      todo &= ~same;
    }
    wave_sync();
    PPROF_ADD(26, tcg);
    {
      PPROF_T0(tce);
      CollEnt cv;
#ifdef SWIM_PHASE_PROF
      uint32_t probes = 0;
      CollEnt* col = coll_ensure_wave(c, r, grp != 0, g.gossiper, lane, cv, &probes);
      PPROF_CNT(31, (unsigned long long)probes);  // probe rounds of the wave
#else
      CollEnt* col = coll_ensure_wave(c, r, grp != 0, g.gossiper, lane, cv);
#endif
      PPROF_ADD(27, tce);
      PPROF_CNT(30, (unsigned long long)__popcll(__ballot(grp != 0)));  // leaders
      // inline collectors: each leader runs its adds in registers (one store at the end); a run that
      // needs a second interval, and every spilled collector, goes on to the staged pass with the
      // lanes it has left (rest).  A cleared collector takes its adds here too; while states older
      // than the clear are in the slab its accepted lanes look their state up in (c) (relook)
      const bool relook_grp = col && (cv.meta & COLL_CLEARED) && pre;
      uint64_t rest = 0;
      if (col && (cv.meta & 7u) == COLL_SPILLED) {
        rest = grp;
      } else if (col) {
        const CollEnt v0 = cv;
        for (uint64_t mm = grp; mm; mm &= mm - 1) {
          const uint32_t j = (uint32_t)__ffsll((unsigned long long)mm) - 1;
          const int a = coll_add_inline(cv, L.iP[j]);
          if (a < 0) {
            rest = mm;
            break;
          }
          L.iS[j] = (uint32_t)a;
        }
        if (!rest && (cv.lo != v0.lo || cv.hi != v0.hi || cv.meta != v0.meta)) *col = cv;
      }
      wave_sync();
      // the staged pass, one collector at a time with the whole wave: its intervals into LDS, the
      // leader's adds there, the result back (coll_place)
      for (uint64_t lm = __ballot(rest != 0); lm; lm &= lm - 1) {
        const uint32_t l = (uint32_t)__ffsll((unsigned long long)lm) - 1;
        const uint64_t rm = rdlane64(rest, l);
        CollEnt* e = reinterpret_cast<CollEnt*>(rdlane64(reinterpret_cast<uint64_t>(col), l));
        const uint32_t meta = rdlane(cv.meta, l);
        const bool spilled = (meta & 7u) == COLL_SPILLED;
        const uint32_t* blk = spilled ? coll_block(c, meta) : nullptr;
        const uint32_t n0 = spilled ? rdlane(gload(blk), 0) : 1u;
        if (COOP_STAGE && n0 + (uint32_t)__popcll(rm) <= 64u) {
          // small collectors (nearly all): interval q in lane q's registers, each add a ballot for
          // its floor, register reads of the neighbours and a one-lane shift across the wave
          PPROF_T0(tsr);
          uint32_t vlo = 0, vhi = 0;
          if (spilled) {
            if (lane < n0) {
              const uint2 t = gload(reinterpret_cast<const uint2*>(blk + 4) + lane);
              vlo = t.x;
              vhi = t.y;
            }
          } else if (lane == 0) {
            vlo = rdlane(cv.lo, l);
            vhi = rdlane(cv.hi, l);
          }
          uint32_t n = n0, maxn = n0, res = 0;
          bool seg = false;
          for (uint64_t mm = rm; mm; mm &= mm - 1) {
            const uint32_t j = (uint32_t)__ffsll((unsigned long long)mm) - 1;
            const uint32_t x = rdlane(g.seq, j);
            const uint64_t le = __ballot(lane < n && vlo <= x);
            const int fl = le ? 63 - __clzll((long long)le) : -1;
            const uint32_t fhi = rdlane(vhi, fl < 0 ? 0u : (uint32_t)fl);
            if (fl >= 0 && x <= fhi) continue;  // held already (res stays 0)
            const uint32_t ce = (uint32_t)(fl + 1);
            const uint32_t clo = rdlane(vlo, ce < n ? ce : 0u), chi = rdlane(vhi, ce < n ? ce : 0u);
            const bool nf = fl >= 0 && (int64_t)x - 1 == (int64_t)fhi;
            const bool nc = ce < n && (int64_t)x + 1 == (int64_t)clo;
            if (nf && nc) {  // x joins its two neighbours: the lanes after ce move down one
              const uint32_t dlo = wave_from_next(vlo), dhi = wave_from_next(vhi);
              if (lane == (uint32_t)fl) vhi = chi;
              if (lane >= ce) { vlo = dlo; vhi = dhi; }
              n--;
            } else if (nf) {
              if (lane == (uint32_t)fl) vhi = x;
            } else if (nc) {
              if (lane == ce) vlo = x;
            } else {  // a new interval at ce: the lanes from ce on move up one
              const uint32_t ulo = wave_from_prev(vlo), uhi = wave_from_prev(vhi);
              if (lane > ce) { vlo = ulo; vhi = uhi; }
              if (lane == ce) { vlo = x; vhi = x; }
              n++;
            }
            if (lane == j) res = 1;
            seg |= n >= 2 && n > (uint32_t)c.seg_threshold;
            maxn = max(maxn, n);
          }
          if ((rm >> lane) & 1ull) L.iS[lane] = res;
          uint32_t* dst = nullptr;
          if (lane == l) {
            if (seg) c.seg_flag[i] = 1;
            dst = coll_place(c, e, meta, n, maxn, rdlane(vlo, 0), rdlane(vhi, 0));
          }
          dst = reinterpret_cast<uint32_t*>(rdlane64(reinterpret_cast<uint64_t>(dst), l));
          if (dst && lane < n) reinterpret_cast<uint2*>(dst + 4)[lane] = make_uint2(vlo, vhi);
          wave_sync();
          PPROF_ADD(38, tsr);
          PPROF_CNT(39, 1ull);
          continue;
        }
        if (!COOP_STAGE || n0 + (uint32_t)__popcll(rm) > COOP_LIV) {  // beyond the staging area
          if (!COOP_STAGE || !spilled) {  // coll_add one by one
            if (lane == l) {
              if (!spilled) *e = cv;
              for (uint64_t mm = rm; mm; mm &= mm - 1) {
                const uint32_t j = (uint32_t)__ffsll((unsigned long long)mm) - 1;
                L.iS[j] = coll_add(c, e, L.iP[j], &c.seg_flag[i]) ? 1u : 0u;
              }
            }
          } else {  // in place in its block, each add by the whole wave
            for (uint64_t mm = rm; mm; mm &= mm - 1) {
              const uint32_t j = (uint32_t)__ffsll((unsigned long long)mm) - 1;
              const int a = coll_add_wave(c, e, L.iP[j], lane, [] { wave_sync(); }, &c.seg_flag[i]);
              if (lane == 0) L.iS[j] = (uint32_t)a;
            }
          }
          wave_sync();
          continue;
        }
        PPROF_T0(tsi);
        PPROF_CNT(35, 1ull);
        PPROF_CNT(36, (unsigned long long)n0);
        if (spilled) {
          const uint2* giv = reinterpret_cast<const uint2*>(blk + 4);
          for (uint32_t q2 = lane; q2 < n0; q2 += 64) siv[q2] = gload(giv + q2);
        } else if (lane == 0) {
          siv[0] = make_uint2(rdlane(cv.lo, l), rdlane(cv.hi, l));
        }
        wave_sync();
        PPROF_ADD(32, tsi);
        PPROF_T0(tsa);
        uint32_t n = n0;
        uint32_t* dst = nullptr;
        uint32_t moved = 0;
        // the leader's adds, made by the whole wave (coll_add_lds_wave: the moves 64 at a time)
        uint32_t maxn = n;
        bool seg = false;
        for (uint64_t mm = rm; mm; mm &= mm - 1) {
          const uint32_t j = (uint32_t)__ffsll((unsigned long long)mm) - 1;
          const int a = coll_add_lds_wave(siv, n, L.iP[j], lane, [] { wave_sync(); }, &moved);
          if (lane == 0) L.iS[j] = (uint32_t)a;
          seg |= a && n >= 2 && n > (uint32_t)c.seg_threshold;
          maxn = max(maxn, n);
        }
        wave_sync();
        if (lane == l) {
          if (seg) c.seg_flag[i] = 1;
          dst = coll_place(c, e, meta, n, maxn, siv[0].x, siv[0].y);
        }
        PPROF_CNT(37, (unsigned long long)moved);
        (void)moved;
        PPROF_ADD(33, tsa);
        PPROF_T0(tsw);
        n = rdlane(n, l);
        dst = reinterpret_cast<uint32_t*>(rdlane64(reinterpret_cast<uint64_t>(dst), l));
        if (dst) {
          uint2* div = reinterpret_cast<uint2*>(dst + 4);
          for (uint32_t q2 = lane; q2 < n; q2 += 64) div[q2] = siv[q2];
        }
        wave_sync();
        PPROF_ADD(34, tsw);
      }
      wave_sync();
      if (relook_grp)
        for (uint64_t mm = grp; mm; mm &= mm - 1) {
          const uint32_t j = (uint32_t)__ffsll((unsigned long long)mm) - 1;
          if (L.iS[j] == 1u) L.iS[j] = 3u;
        }
      PPROF_ADD(28, tce);
    }
    wave_sync();
    // the next chunk's collector slots, warmed while (b) and (c) run (its messages are in by now)
#if COOP_PIPE
    const uint32_t warm = more && q + 64 < k ? cbase[hash32(gn.gossiper) & (c.hcap - 1)].key : 0u;
#else
    const uint32_t warm = 0u;
#endif
    PPROF_ADD(13, tca);
    PPROF_T0(tcb);
    const uint32_t fl = L.iS[lane];
    const bool accepted = fl == 1u || fl == 3u;
    const bool relook = fl == 3u;  // accepted by a cleared collector: its state is looked up at its turn
    const bool full = (valid && !coop) || fl == 2u;  // the chain's onGossipReq, at its turn
    // (b) receipts; the records that cannot change the view
    const bool user = g.status() >= SWIM_GOSSIP_USER;
    // the subject's cell is loaded before the receipt mark's slot read: both in flight at once
    const uint64_t cell = accepted && !user ? cell_get(c, r, g.subject) : 0ull;
    if (accepted) receipt_mark(c, r, g.gossiper, g.seq);
    bool noop = false;
    if (accepted && !user) {
      if (c.n_ns && !c.ns_rel[(size_t)c.ns[r] * c.n_ns + c.ns[g.subject]]) {
        noop = true;
      } else {
        const bool present = c_has(cell, B_IN_TABLE);
        const uint32_t st0 = c_status(cell);
        noop = !(present && st0 == SWIM_LEAVING) && !is_overrides(g.status(), g.inc(), present, st0, c_inc(cell));
      }
    }
    bool skip = accepted && noop && !relook;
    // (a lane that may change its subject's record: an accepted non-no-op one, or one taking the
    // chain's onGossipReq or a lookup)
    for (uint64_t mm = __ballot(((accepted && !noop) || full || relook) && !user); mm; mm &= mm - 1) {
      const uint32_t j = (uint32_t)__ffsll((unsigned long long)mm) - 1;
      const uint32_t sj = rdlane(g.subject, j);
      if (lane > j && !user && g.subject == sj) skip = false;
    }
    // (c) positions and the serial steps, in rank order.  Each state is written (and indexed) as soon
    // as its position is known, before any later lane's onGossipReq may look the slab up (gix_find
    // after a collector clear rebuilds the index from the slab)
    const uint64_t accm = __ballot(accepted);
    const uint64_t serm = __ballot((accepted && !skip) || full);
    PPROF_ADD(14, tcb);
    PPROF_CNT(6, (unsigned long long)__popcll(serm));  // lanes taking a serial step
    PPROF_CNT(7, (unsigned long long)__popcll(accm));  // accepted lanes
    PPROF_CNT(47, (unsigned long long)__popcll(__ballot(full)));  // lanes taking the chain's onGossipReq
    PPROF_T0(tcc);
    const uint64_t below_me = (1ull << lane) - 1;
    if (pre && __ballot(full || relook) && !__builtin_amdgcn_readfirstlane(m.gix_valid)) {
      PPROF_T0(tgr);
      gix_rebuild_wave(c, m, r, slab, len, lane);
      PPROF_CNT(53, 1ull);
      PPROF_ADD(54, tgr);
    }
    GossipDev ns;
    ns.gossiper = g.gossiper; ns.seq = g.seq; ns.subject = g.subject; ns.status = g.status(); ns.inc = g.inc();
    ns.inf_period = period;
    ns.inf[0] = g.from;
#pragma unroll
    for (int x = 1; x < GINF; ++x) ns.inf[x] = NONE;
    unsigned long long fullacc = 0;
    uint64_t done = 0;
    for (uint64_t mm = serm;;) {
      const uint32_t jn = mm ? (uint32_t)__ffsll((unsigned long long)mm) - 1 : 64u;
      const uint64_t below = jn == 64u ? ~0ull : ((1ull << jn) - 1);
      const uint64_t blk = accm & ~serm & below & ~done;  // no-op lanes before the next serial one
      if (blk) {
        PPROF_T0(tbk);
        uint32_t pos = NONE;
        if ((blk >> lane) & 1ull) {
          const uint32_t p = len + (uint32_t)__popcll(blk & below_me);
          if (p < c.gcap) {
            pos = p;
            slab.put(p, ns);
          } else {
            set_err(c, ERR_SLAB);
          }
        }
        len = min(len + (uint32_t)__popcll(blk), c.gcap);
        if (__builtin_amdgcn_readfirstlane(m.gix_valid)) {  // (only after a collector clear needed the index)
          // the block's states noted in the index together (gix_note_at for every lane at once; at
          // half load the index is dropped, to be rebuilt by the next lookup)
          const uint32_t nput = (uint32_t)__popcll(__ballot(pos != NONE));
          const uint32_t used0 = __builtin_amdgcn_readfirstlane(m.gix_used);
          PPROF_CNT(48, (unsigned long long)nput);
          if (2 * (used0 + nput) >= c.gix_mask + 1) {
            if (lane == 0) m.gix_valid = 0;
          } else {
            const bool took = pos != NONE && gix_put_atomic(gix_of(c, r), c.gix_mask, __builtin_amdgcn_readfirstlane(m.gix_base),
                                                            len, g.gossiper, g.seq,
                                                            __builtin_amdgcn_readfirstlane(m.gix_base) + pos);
            const uint32_t nt = (uint32_t)__popcll(__ballot(took));
            if (lane == 0) m.gix_used = used0 + nt;
          }
        }
        done |= blk;
        wave_sync();
        PPROF_ADD(49, tbk);
      }
      if (!mm) break;
      PPROF_T0(tsr);
      uint32_t nl = 0;
      if (lane == jn) {
        gsr.len = len;
        if (full) {
          fullacc += on_gossip_req(c, r, m, slab, g) ? 1u : 0u;
        } else if (relook) {
          gossip_accepted(c, r, m, slab, g, true);
        } else if (len >= c.gcap) {
          set_err(c, ERR_SLAB);
        } else {
          slab.put(len, ns);
          gsr.len = len + 1;
          gix_note(c, m, r, ns.gossiper, ns.seq);
          if (user)  // sink.next(gossip.message()) (:209): listen() subscribers
            emit(c, r, g.gossiper, SWIM_EV_GOSSIP, SWIM_PHASE_GOSSIP, m.ev_minor++, g.subject);
          else if (update_membership(c, r, g.subject, g.status(), g.inc(), R_GOSSIP, SWIM_PHASE_GOSSIP))
            apply_alive(c, r, g.subject, g.inc(), R_GOSSIP, SWIM_PHASE_GOSSIP);
        }
        nl = gsr.len;
      }
      len = rdlane(nl, jn);
      done |= 1ull << jn;
      mm &= mm - 1;
      wave_sync();
#ifdef SWIM_PHASE_PROF
      if (rdlane(full || relook ? 1u : 0u, jn)) PPROF_ADD(50, tsr); else PPROF_ADD(51, tsr);
#endif
    }
    PPROF_ADD(15, tcc);
    acc += (accepted ? 1ull : 0ull) + fullacc;  // (per lane: the caller sums the wave)
    if (lane == 0) gsr.len = len;
    sink ^= warm;
    wave_sync();
  }
  if (sink == 0x5bd1e995u && k == 0x7fffffffu) set_err(c, 0u);  // keeps the warming loads; sets no bit
  return acc;
}

// The big inboxes of at least coop_min messages, before k_gossip_deliver (a kernel of its own: the
// whole-wave delivery's registers do not weigh on the main delivery kernel): a wave per inbox,
// grid-stride over big_list — rank, deliver_coop, the inbox pages back to the pool, msg_cnt = 0; the
// main kernel then finds the inbox empty and does the receiver's pingMembers inserts and SYNC
// collection as for any big inbox.  prof as k_gossip_deliver's.
#ifndef COOP_OCC
#define COOP_OCC 2  // blocks per CU the whole-wave delivery kernel is compiled for (3 / 4 spill: 0.44 / 0.53 ms vs 0.41)
#endif
__global__ void __launch_bounds__(DLV_BLOCK, COOP_OCC) k_deliver_coop(KP, unsigned long long* prof) {
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  __shared__ BigLds s_big[DLV_WAVES];
  __shared__ uint2 s_iv[DLV_WAVES][COOP_LIV];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long acc = 0;
  uint32_t nmsg = 0, nfresh = 0;
  if (b.k->msg_total != 0) {
    const uint32_t nbig = b.k->big_cnt;
    for (uint32_t x = __builtin_amdgcn_readfirstlane(blockIdx.x * DLV_WAVES + wv); x < nbig; x += gridDim.x * DLV_WAVES) {
      const uint32_t i = b.big_list[x];
      const uint32_t r = c.lo + i;
      const uint32_t k = min(b.msg_cnt[i], b.pg_max * 64u);  // (beyond the page table: ERR_INBOX is set)
      if (k < b.coop_min) continue;  // (wave-uniform) the main kernel's lane chains take it
      uint32_t* pt = b.pg_tab + (size_t)i * b.pg_max;
      bool pages_ok = true;
      for (uint32_t pg = lane; pg < (k + 63) / 64; pg += 64) pages_ok &= pt[pg] < b.pg_cap;
      pages_ok = __ballot(!pages_ok) == 0;
      wave_sync();
      if (lane == 0) b.msg_cnt[i] = 0;
      if (c.up[r] && pages_ok) {
        rank_big_inbox(c, b, i, k, lane, s_big[wv], true);
        nmsg += lane == 0 ? k : 0u;
        acc += deliver_coop(c, b, i, k, lane, s_big[wv], s_iv[wv], nfresh);
      }
      wave_sync();
      for (uint32_t pg = lane; pg < (k + 63) / 64; pg += 64)
        if (pg) pt[pg] = NONE;  // (page 0 is the receiver's own)
    }
  }
  wave_stat_add(c, ST_GOSSIP_ACCEPTED, acc);
  if (prof) {
    const unsigned long long a0 = wave_sum(nmsg), a1 = wave_sum(nfresh), a2 = wave_sum(acc);
    if (lane == 0 && (a0 | a1 | a2)) {
      atomicAdd(prof, a0);
      atomicAdd(prof + 1, a1);
      atomicAdd(prof + 2, a2);
    }
  }
}

__device__ unsigned long long deliver_big_batch(const Ctx& c, const Ctx& cs, const Bufs& b, const uint32_t* list,
                                                uint32_t nb, uint32_t lane, int collect, BigLds& L,
                                                unsigned long long& nsync, uint32_t& nmsg, uint32_t& nfresh) {
  // 1. rank every inbox of the batch; lane j keeps receiver j's message count (0: nothing to
  //    deliver) and the count of inbox pages to hand back
  PPROF_T0(tp0);
  PPROF_CNT(4, 1ull);
  PPROF_CNT(5, (unsigned long long)nb);
  uint32_t my_k = 0, my_pages = 0;
  for (uint32_t j = 0; j < nb; ++j) {
    const uint32_t i = list[j];
    const uint32_t r = c.lo + i;
    const uint32_t k_all = b.msg_cnt[i];
    wave_sync();
    if (lane == 0) b.msg_cnt[i] = 0;
    // messages beyond the page table were never written (ERR_INBOX is set)
    const uint32_t k = min(k_all, b.pg_max * 64u);
    const uint32_t* pt = b.pg_tab + (size_t)i * b.pg_max;
    bool pages_ok = true;
    // a page the pool could not give holds NONE or PG_FAILED (ERR_PAGES / ERR_INBOX are set)
    for (uint32_t pg = lane; pg < (k + 63) / 64; pg += 64) pages_ok &= pt[pg] < b.pg_cap;
    pages_ok = __ballot(!pages_ok) == 0;
    const bool go = c.up[r] && k && pages_ok;
    if (go) {
      rank_big_inbox(c, b, i, k, lane, L);
      nmsg += lane == 0 ? k : 0u;
    }
    if (lane == j) {
      my_k = go ? k : 0;  // (an inbox of >= coop_min messages was delivered by k_deliver_coop: k = 0 here)
      my_pages = (k + 63) / 64;
    }
  }
  wave_sync();
  PPROF_ADD(0, tp0);
  PPROF_T0(tp1);
  // 2. the onGossipReq chains, lane j for receiver j
#ifdef SWIM_PHASE_PROF
  if (lane < nb && my_k) {
    atomicMax(&g_dbg[10], (unsigned long long)my_k);  // the longest chain of the launches
    atomicAdd(&g_dbg[11], (unsigned long long)my_k);  // messages walked by the chains
  }
  {
    uint32_t mx = lane < nb ? my_k : 0u;  // the wave's longest chain (its time is that chain's)
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
    PPROF_CNT(12, (unsigned long long)mx);
  }
#endif
  unsigned long long acc = 0;
  if (lane < nb && my_k) {
    const uint32_t i = list[lane], r = c.lo + i;
    const uint32_t* pt = b.pg_tab + (size_t)i * b.pg_max;
    MemberDev& m = mem(c, r);
    m.ev_minor = 0;
    m.fetch_ctr = 0;
    const SlabRef slab = slab_of(c, r);
    // the next message (and its collector slot) is fetched while the current one is processed: the
    // chain's own dependent round trips are the cost of a big inbox
    auto fetch = [&](uint32_t q) -> GMsgFull {
      uint32_t jq = b.pg_perm[(size_t)pt[q >> 6] * 64 + (q & 63)];
      if (jq >= my_k) {  // a hole: only after an inbox overflow (ERR_MSGS is set)
        set_err(c, ERR_MSGS);
        jq = q;
      }
      return b.pg_msgs[(size_t)pt[jq >> 6] * 64 + (jq & 63)];
    };
    const CollEnt* cbase = c.coll + (size_t)i * c.hcap;
    uint32_t sink = 0;
    GMsgFull next = fetch(0);
    for (uint32_t q = 0; q < my_k; ++q) {
      const GMsgFull g = next;
      if (q + 1 < my_k) {
        next = fetch(q + 1);
        sink ^= warm_gossip_req(c, r, cbase, next);
      }
      nfresh += g.dup() ? 0u : 1u;
      if (on_gossip_req(c, r, m, slab, g)) acc++;
    }
    if (sink == 0x5bd1e995u && my_k == 0x7fffffffu) set_err(c, 0u);  // keeps the warming loads; sets no bit
  }
  wave_sync();
  PPROF_ADD(1, tp1);
  PPROF_T0(tp2);
  // 3. per receiver: the inbox pages go back to the pool (the pool itself restarts every tick) and
  //    the phase's pingMembers inserts run (wave-cooperative, receiver by receiver); then phase D's
  //    SYNC collection of the batch's receivers, lane j for receiver j (member-local, as in the
  //    small-inbox path: each reads only its own lists, schedule and FD-SYNC queue)
  for (uint32_t j = 0; j < nb; ++j) {
    const uint32_t i = list[j], r = c.lo + i;
    const uint32_t np = rdlane(my_pages, j);
    for (uint32_t pg = lane; pg < np; pg += 64)
      if (pg) b.pg_tab[(size_t)i * b.pg_max + pg] = NONE;  // (page 0 is the receiver's own)
#ifdef SWIM_PHASE_PROF
    {  // inserts applied: count, receivers, their lists' lengths, the largest batch, the time
      const uint32_t kk = __builtin_amdgcn_readfirstlane(mem(c, r).ins_rank);
      if (kk) {
        PPROF_CNT(41, (unsigned long long)kk);
        PPROF_CNT(43, 1ull);
        PPROF_CNT(44, (unsigned long long)__builtin_amdgcn_readfirstlane(mem(c, r).ping_len));
        if (lane == 0) atomicMax(&g_dbg[42], (unsigned long long)kk);
      }
      PPROF_T0(tin);
      apply_ins_batch<64, false>(c, r, lane, L.iP, L.iS, L.iR);
      PPROF_ADD(45, tin);
    }
#else
    apply_ins_batch<64, false>(c, r, lane, L.iP, L.iS, L.iR);
#endif
  }
  PPROF_T0(tcol);
  if (lane < nb && collect) nsync += sync_collect_member(cs, b, c.lo + list[lane]);
  PPROF_ADD(46, tcol);
  PPROF_ADD(2, tp2);
  return acc;
}

// Gossip delivery (phase C) for the round's inboxes, then the pingMembers inserts of every receiver
// (a viewer's ADDED events of the phase all come from the one thread / wave that delivered to it),
// then phase D's SYNC collection of every member, each right after its own deliveries and inserts
// (nothing else in the gossip phase touches what sync_collect_member reads: the member's own lists,
// schedule and fd_sync queue).  First the big inboxes, a wave each, grid-stride over big_list;
// then each workgroup's blocks of 256 members: small inboxes thread per receiver, their inserts by
// the workgroup, the collection of members whose inbox was not big.
// prof (sampled launches only): {inbox messages delivered, of which not provable duplicates, accepted}
__global__ void __launch_bounds__(DLV_BLOCK) k_gossip_deliver(KP, int collect, unsigned long long* prof) {
  const Ctx c = pctx(P, T);
  const Ctx cs = pctx_sync(P, T);
  const Bufs b = P->b;
  __shared__ uint64_t s_key[DLV_SORT][DLV_BLOCK];
  __shared__ uint8_t s_ix[DLV_SORT][DLV_BLOCK];
  __shared__ BigLds s_big[DLV_WAVES];
  __shared__ uint32_t s_ins[DLV_BLOCK];
  __shared__ uint32_t s_nins;
  __shared__ uint32_t s_iP[DLV_BLOCK], s_iS[DLV_BLOCK], s_iR[DLV_BLOCK];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t t32 = (uint32_t)T;
  // the schedule words of this thread's first member, loaded beside the inbox flag (nothing in the
  // gossip phase changes them: k_fd set its mflag bits, the SYNC collection below consumes them)
  const uint32_t i_first = blockIdx.x * DLV_BLOCK + tid;
  uint32_t sn_first = NONE, fl_first = 0;
  if (collect && i_first < c.nl) {
    sn_first = c.sync_next[i_first];
    fl_first = c.mflag[i_first];
  }
  const bool any = b.k->msg_total != 0;  // else no receiver has an inbox
  unsigned long long acc = 0, nsync = 0;
  uint32_t nmsg = 0, nfresh = 0;
  if (any) {  // big inboxes in batches of up to 64 per wave, spread over every wave of the grid
    const uint32_t nbig = b.k->big_cnt;
    const uint32_t nw = gridDim.x * DLV_WAVES;
    const uint32_t bsz = min(64u, max(1u, (nbig + nw - 1) / nw));
    for (uint32_t x = __builtin_amdgcn_readfirstlane((blockIdx.x * DLV_WAVES + wv) * bsz); x < nbig; x += nw * bsz)
      acc += deliver_big_batch(c, cs, b, b.big_list + x, min(bsz, nbig - x), lane, collect, s_big[wv], nsync, nmsg,
                               nfresh);
  }
  PPROF_T0(tp3);
  for (uint32_t base = blockIdx.x * DLV_BLOCK; base < c.nl; base += gridDim.x * DLV_BLOCK) {
    if (tid == 0) s_nins = 0;
    __syncthreads();
    const uint32_t i = base + tid;
    // a big inbox's receiver is owned by its wave for the whole kernel (big_tick is stable; msg_cnt
    // is not: the wave zeroes it)
    const bool big = any && i < c.nl && b.big_tick[i] == t32;
    if (any && i < c.nl && !big) {
      const uint32_t k = b.msg_cnt[i];
      const uint32_t r = c.lo + i;
      if (k != 0) {
        // a small inbox fits its first page (k <= DLV_SORT < 64): the receiver's own, page i
        b.msg_cnt[i] = 0;
        const uint32_t pid = i;
        if (!c.up[r]) {
        } else if (pid >= b.pg_cap) {  // NONE or PG_FAILED: the page pool ran dry (ERR_PAGES is set)
          set_err(c, ERR_PAGES);
        } else {
          const GMsgFull* a = b.pg_msgs + (size_t)pid * 64;
          for (uint32_t q = 0; q < k; ++q) {
            const uint64_t kx = msg_key(c, a[q]);  // keys are unique
            int32_t j = (int32_t)q - 1;
            while (j >= 0 && s_key[j][tid] > kx) {
              s_key[j + 1][tid] = s_key[j][tid];
              s_ix[j + 1][tid] = s_ix[j][tid];
              --j;
            }
            s_key[j + 1][tid] = kx;
            s_ix[j + 1][tid] = (uint8_t)q;
          }
          nmsg += k;
          acc += deliver_sorted(c, r, a, k, &s_ix[0][tid], DLV_BLOCK, nfresh);
          if (c.mem[i].ins_rank) s_ins[atomicAdd(&s_nins, 1u)] = r;
        }
      }
    }
    __syncthreads();
    const uint32_t nv = s_nins;
    for (uint32_t q = 0; q < nv; ++q) apply_ins_batch<DLV_BLOCK, true>(c, s_ins[q], tid, s_iP, s_iS, s_iR);
    if (collect && i < c.nl && !big)
      nsync += i == i_first ? sync_collect_pre(cs, b, c.lo + i, sn_first, fl_first) : sync_collect_member(cs, b, c.lo + i);
  }
  PPROF_ADD(3, tp3);
  wave_stat_add(c, ST_GOSSIP_ACCEPTED, acc);
  wave_stat_add(cs, ST_SYNCS, nsync);
  if (prof) {
    const unsigned long long a0 = wave_sum(nmsg), a1 = wave_sum(nfresh), a2 = wave_sum(acc);
    if ((tid & 63) == 0 && (a0 | a1 | a2)) {
      atomicAdd(prof, a0);
      atomicAdd(prof + 1, a1);
      atomicAdd(prof + 2, a2);
    }
  }
}


// ------------------------------------------------------------------------------- phase D
// member v's MembershipConfig.seedMembers (MembershipProtocolImpl.java:120-130, cleanUpSeedMembers
// :171-190): its own list (swim_set_member_seeds) or the engine-wide one (swim_set_seeds)
__device__ __forceinline__ bool own_seeds(const Ctx& c, uint32_t v) { return c.mseed_own && c.mseed_own[v]; }
__device__ __forceinline__ const uint32_t* seeds_of(const Ctx& c, uint32_t v, uint32_t& ns) {
  if (!own_seeds(c, v)) {
    ns = c.n_seeds;
    return c.seeds;
  }
  ns = c.mseed_off[v + 1] - c.mseed_off[v];
  return c.mseed + c.mseed_off[v];
}
__device__ inline bool is_seed_of(const Ctx& c, uint32_t v, uint32_t x) {
  if (!own_seeds(c, v)) return c.is_seed[x] != 0;
  for (uint32_t k = c.mseed_off[v]; k < c.mseed_off[v + 1]; ++k)
    if (c.mseed[k] == x) return true;
  return false;
}

// selectSyncAddress (MembershipProtocolImpl.java:461-472): uniform over seeds U otherMembers by
// seeded rejection sampling.
__device__ inline uint32_t select_sync_address(const Ctx& c, uint32_t v) {
  const MemberDev& m = mem(c, v);
  const uint32_t* a = aux_row(c, v);
  // seed addresses exclude the local one (cleanUpSeedMembers :171-190)
  uint32_t count = m.members_size - 1, ns = 0;
  const uint32_t* sl = seeds_of(c, v, ns);
  for (uint32_t i = 0; i < ns; ++i) {
    uint32_t s = sl[i];
    if (s != v && dst(c, s) != v && !(a[s] & A_IN_MEMBERS)) count++;
  }
  if (count == 0) return NONE;
  for (uint32_t i = 0; i < SWIM_SYNC_SELECT_ATTEMPTS; ++i) {
    uint32_t x = next_int(draw(c, v, SWIM_STREAM_SYNC_SELECT, 0, i), c.n);
    if (x != v && ((a[x] & A_IN_MEMBERS) || (is_seed_of(c, v, x) && dst(c, x) != v))) return x;
  }
  uint32_t k = next_int(draw(c, v, SWIM_STREAM_SYNC_SELECT, 1, 0), count);
  for (uint32_t x = 0; x < c.n; ++x)
    if (x != v && ((a[x] & A_IN_MEMBERS) || (is_seed_of(c, v, x) && dst(c, x) != v))) {
      if (k == 0) return x;
      --k;
    }
  return NONE;
}

// SyncReq.flags: bits 0..2 below; bits 8..31 the number of records the message carries (the
// sender's table size when the message is prepared: the count syncMembership iterates, :491-509)
// RQ_PARKED: a delayed message (content in park slot .snap, sent in tick .pad); RQ_ACK: in the delay
// queue, a SYNC_ACK (else a SYNC)
// RQ_DEFER: a SYNC_ACK of this tick that k_ack_delay parked (its SYNC_ACK sub-phase skips it)
// RQ_PHANTOM: a deferred SYNC_ACK whose waits completed (PAck): it takes the place of a SYNC in the
// acker's inbox, merges nothing and gets its SYNC_ACK like every SYNC of the tick (.from = the ack's
// receiver, .pad = the PAck's seq); with RQ_DEFER, in tx_reqs: a marker telling the shard of the
// ack's receiver, before its SYNC merges, that an ack will come (SF_SENT | SF_MULTI)
// RQ_WAIT: a SYNC whose Monos are still running (a PAck holds its SYNC_ACK)
enum : uint32_t { RQ_INITIAL = 1, RQ_OUTFAIL = 2, RQ_DELIVERED = 4, RQ_PHANTOM = 8, RQ_PARKED = 16, RQ_ACK = 32,
                  RQ_DEFER = 64, RQ_WAIT = 128, RQ_RECS_SHIFT = 8 };

// per-member SYNC roles of the tick (Bufs.sflag)
enum : uint32_t {
  SF_SENT_LOCAL = 1,  // sent a SYNC delivered to a receiver on this shard (its row is read as content)
  SF_SENT = 2,        // sent a delivered SYNC (it may be merged into in the SYNC_ACK sub-phase)
  SF_RECV = 4,        // received a SYNC (its row is merged into in the SYNC sub-phase)
  SF_MULTI = 8,       // sent two or more SYNCs: more than one SYNC_ACK may come back
};
constexpr uint32_t SF_BITS = 4, SF_MASK = (1u << SF_BITS) - 1;  // sflag = tick << SF_BITS | SF_*
__device__ inline uint32_t snap_take(const Ctx& c, const Bufs& b, uint32_t i) {
  const uint32_t par = (uint32_t)(c.T & 1);
  const uint32_t slot = atomicAdd(&b.snap_cnt[par], 1u);
  if (slot >= b.snap_cap) { set_err(c, ERR_SNAP); return NONE; }
  b.snap_list[par * b.snap_cap + slot] = i;
  return slot;
}
// add SF_* bits to member i's roles this tick; the update that completes {SENT, RECV} claims the
// snapshot slot of i: its row is read as message content while its own merges change it (the SYNC
// it sent carries its table when the SYNC was prepared, :485-489; the SYNC_ACK it sends carries its
// table after its SYNC merges).  k_sync_classify fills the slot from the units of the SYNCs i
// receives (they stream i's row before any merge); k_sync_apply copies i's row again, into a slot
// of its own for the SYNC_ACK content, only when i's SYNC merges changed it.
// (old: the caller's guess of the word, loaded early; a stale guess only costs a CAS retry)
__device__ inline void sflag_set_from(const Ctx& c, const Bufs& b, uint32_t i, uint32_t bits, uint32_t old) {
  const uint32_t t3 = (uint32_t)c.T << SF_BITS;
  for (;;) {
    const uint32_t base = (old & ~SF_MASK) == t3 ? old : t3;
    const uint32_t nw = base | bits;
    if (nw == old) return;
    const uint32_t prev = atomicCAS(&b.sflag[i], old, nw);
    if (prev == old) {
      if ((nw & (SF_SENT | SF_RECV)) == (SF_SENT | SF_RECV) && (base & (SF_SENT | SF_RECV)) != (SF_SENT | SF_RECV)) {
        const uint32_t slot = snap_take(c, b, i);
        b.snap_idx[i] = slot;
        b.ack_snap[i] = slot;
      }
      return;
    }
    old = prev;
  }
}
// sflag_set_from split in two, so that its CAS is in flight together with other atomics: sflag_cas
// issues one attempt (none when the bits are already set), sflag_done finishes the update — the slot
// claim on success, the retry loop after a lost race
struct SfCas {
  uint32_t old, nw, prev;
};
__device__ __forceinline__ SfCas sflag_cas(const Ctx& c, const Bufs& b, uint32_t i, uint32_t bits, uint32_t old) {
  const uint32_t t3 = (uint32_t)c.T << SF_BITS;
  const uint32_t base = (old & ~SF_MASK) == t3 ? old : t3;
  SfCas r{old, base | bits, old};
  if (r.nw != old) r.prev = atomicCAS(&b.sflag[i], old, r.nw);
  return r;
}
__device__ __forceinline__ void sflag_done(const Ctx& c, const Bufs& b, uint32_t i, uint32_t bits, const SfCas& r) {
  if (r.nw == r.old) return;
  if (r.prev != r.old) {
    sflag_set_from(c, b, i, bits, r.prev);
    return;
  }
  const uint32_t t3 = (uint32_t)c.T << SF_BITS;
  const uint32_t base = (r.old & ~SF_MASK) == t3 ? r.old : t3;
  if ((r.nw & (SF_SENT | SF_RECV)) == (SF_SENT | SF_RECV) && (base & (SF_SENT | SF_RECV)) != (SF_SENT | SF_RECV)) {
    const uint32_t slot = snap_take(c, b, i);
    b.snap_idx[i] = slot;
    b.ack_snap[i] = slot;
  }
}
__device__ __forceinline__ void sflag_set(const Ctx& c, const Bufs& b, uint32_t i, uint32_t bits) {
  sflag_set_from(c, b, i, bits, b.sflag[i]);
}
__device__ __forceinline__ bool sflag_has(const Ctx& c, const Bufs& b, uint32_t i, uint32_t bits) {
  const uint32_t f = b.sflag[i];
  return (f & ~SF_MASK) == ((uint32_t)c.T << SF_BITS) && (f & bits) == bits;
}

constexpr uint32_t SY_INLINE = 4;
struct SyInbox {  // the SYNC (d2 = 0) or SYNC_ACK (d2 = 1) sub-phase's items and inboxes
  SyncReq* items;
  uint32_t* total;
  uint32_t* cnt;
  uint32_t* recv;
  uint32_t* recv_cnt;
  uint32_t* inl;
  uint32_t* tab;
  uint32_t* pool;
  uint32_t* pg;
};
__device__ __forceinline__ SyInbox sy_inbox(const Bufs& b, int d2) {
  SyInbox x;
  if (!d2) {
    x.items = b.reqs; x.total = &b.k->req_total; x.cnt = b.req_cnt; x.recv = b.req_recv;
    x.recv_cnt = &b.k->req_recv_cnt; x.inl = b.rq_inl; x.tab = b.rq_tab; x.pool = b.rq_pool; x.pg = &b.k->req_pg;
  } else {
    x.items = b.acks; x.total = &b.k->ack_total; x.cnt = b.ack_cnt; x.recv = b.ack_recv;
    x.recv_cnt = &b.k->ack_recv_cnt; x.inl = b.ack_inl; x.tab = b.ack_tab; x.pool = b.ack_pool; x.pg = &b.k->ack_pg;
  }
  return x;
}
// inbox pages of the SYNC sub-phases: allocated by the writer of the page's first slot, awaited by
// the others (the same discipline as the gossip inboxes, inbox_page_alloc / _wait)
__device__ inline uint32_t sy_page_alloc(const Ctx& c, const Bufs& b, const SyInbox& x, uint32_t i, uint32_t pg) {
  if (pg >= b.sy_max) { set_err(c, ERR_REQS); return NONE; }
  uint32_t np = atomicAdd(x.pg, 1u);
  if (np >= b.sy_pool_cap) { set_err(c, ERR_REQS); np = PG_FAILED; }
  __atomic_store_n(x.tab + (size_t)i * b.sy_max + pg, np, __ATOMIC_RELAXED);
  return np == PG_FAILED ? NONE : np;
}
__device__ inline uint32_t sy_page_wait(const Ctx& c, const Bufs& b, const SyInbox& x, uint32_t i, uint32_t pg) {
  if (pg >= b.sy_max) { set_err(c, ERR_REQS); return NONE; }
  const uint32_t* e = x.tab + (size_t)i * b.sy_max + pg;
  for (uint32_t it = 0; it < (1u << 20); ++it) {
    const uint32_t v = __atomic_load_n(e, __ATOMIC_RELAXED);
    if (v != NONE) return v == PG_FAILED ? NONE : v;
    __builtin_amdgcn_s_sleep(2);
  }
  set_err(c, ERR_REQS);
  return NONE;
}

// a delivered SYNC / SYNC_ACK joins its receiver's inbox (the receiver is owned by this shard).
// The item's classification counters start at zero here, before any classify launch adds to them.
// (rsf: a guess of the receiver's sflag word, see sflag_set_from; sbits != 0: the sender's SF_* bits
// of this message, set here from its guessed word sfv, the CAS in flight with the enqueue's atomics)
__device__ inline void enqueue_sync(const Ctx& c, const Bufs& b, int d2, SyncReq q, bool valid, uint32_t rsf,
                                    uint32_t sbits = 0, uint32_t sfv = 0) {
  const SyInbox x = sy_inbox(b, d2);
  uint32_t it = NONE, s = 0, pid = NONE, r = 0;
  if (valid) {
    // the item and the inbox slot are taken together (two independent atomics in flight at once); an
    // item beyond the capacity (ERR_REQS) still takes its slot, as NONE, which readers skip
    r = q.to - c.lo;
    SfCas sc{};
    if (sbits) sc = sflag_cas(c, b, q.from - c.lo, sbits, sfv);
    it = atomicAdd(x.total, 1u);
    s = atomicAdd(&x.cnt[r], 1u);
    if (sbits) sflag_done(c, b, q.from - c.lo, sbits, sc);
    if (it >= b.req_cap) {
      set_err(c, ERR_REQS);
      it = NONE;
    } else {
      q.slot = s;
      x.items[it] = q;
      if (!d2) {
        b.item_total[it] = 0;
        b.rev_total[it] = 0;
      } else {
        b.ack_ctot[it] = 0;
      }
    }
    if (s == 0) {  // the receiver list's entry and the receiver's SF_RECV, both atomics in flight together
      SfCas rc{};
      if (!d2) rc = sflag_cas(c, b, r, SF_RECV, rsf);
      x.recv[atomicAdd(x.recv_cnt, 1u)] = q.to;
      if (!d2) sflag_done(c, b, r, SF_RECV, rc);
    }
    if (s < SY_INLINE) {
      x.inl[(size_t)r * SY_INLINE + s] = it;
      valid = false;  // placed
    } else if (((s - SY_INLINE) & 63) == 0) {
      pid = sy_page_alloc(c, b, x, r, (s - SY_INLINE) >> 6);
    }
  }
  wave_order();
  if (valid && ((s - SY_INLINE) & 63) != 0) pid = sy_page_wait(c, b, x, r, (s - SY_INLINE) >> 6);
  if (valid && pid != NONE) x.pool[(size_t)pid * 64 + ((s - SY_INLINE) & 63)] = it;
}
__device__ __forceinline__ void enqueue_sync(const Ctx& c, const Bufs& b, int d2, SyncReq q, bool valid) {
  enqueue_sync(c, b, d2, q, valid, valid && !d2 ? b.sflag[q.to - c.lo] : 0u);
}

// ---- delayed SYNC / SYNC_ACK (tryDelayOutbound :190-202 on doSync's and onSync's send, :339-357,
// :394-415, and start0's requestResponse :268-276)
__device__ __forceinline__ uint32_t* park_row(const Ctx& c, const Bufs& b, uint32_t slot) {
  return b.park + (size_t)slot * c.n;
}
__device__ inline uint32_t park_alloc(const Ctx& c, const Bufs& b) {
  const int32_t a = atomicSub(&b.park_ctl->avail, 1);
  if (a > 0) return b.park_avail[a - 1];
  const uint32_t i = atomicAdd(&b.park_ctl->bump, 1u);
  if (i < b.park_cap) return i;
  set_err(c, ERR_SDELAY);
  return NONE;
}
// a park slot whose message could not be queued goes back to the pool (reusable from the next tick)
__device__ inline void park_release(const Bufs& b, uint32_t slot) {
  const uint32_t j = atomicAdd(&b.park_ctl->freed, 1u);
  if (j < b.park_cap) b.park_freed[j] = slot;
}
// message q (its content already in park slot q.snap) arrives `k` ticks from now
__device__ inline void park_put(const Ctx& c, const Bufs& b, SyncReq q, uint32_t k, bool ack) {
  q.flags |= RQ_PARKED | (ack ? RQ_ACK : 0u);
  q.pad = (uint32_t)c.T;
  q.content = NONE;
  const uint32_t bk = (uint32_t)(c.T + k) & DQ_MASK;
  const uint32_t i = atomicAdd(&b.sdq_cnt[bk], 1u);
  if (i >= b.sdq_bcap) { set_err(c, ERR_SDELAY); park_release(b, q.snap); return; }
  b.sdq[(size_t)bk * b.sdq_bcap + i] = q;
}
// a delayed SYNC: its content (the sender's row now, before any merge of this tick) is copied by
// k_sync_delay
__device__ inline void park_request(const Ctx& c, const Bufs& b, SyncReq q, uint32_t k) {
  const uint32_t slot = park_alloc(c, b);
  if (slot == NONE) return;
  const uint32_t j = atomicAdd(&b.k->park_jobs, 1u);
  if (j >= b.park_cap) { set_err(c, ERR_SDELAY); park_release(b, slot); return; }
  b.park_jobs[j] = make_uint2(slot, q.from);
  q.snap = slot;
  park_put(c, b, q, k, false);
}

__device__ inline void add_req(const Ctx& c, const Bufs& b, uint32_t v, uint32_t to, uint32_t ordinal, bool initial) {
  MemberDev& m = mem(c, v);
  SyncReq q;
  q.from = v; q.to = to; q.ordinal = ordinal; q.slot = 0;
  q.flags = (initial ? RQ_INITIAL : 0) | (m.table_size << RQ_RECS_SHIFT);
  q.content = NONE; q.snap = NONE; q.pad = 0;
  if (initial) m.init_total++;
  // tryFailOutbound (loss) now; the transport's send after tryDelayOutbound meets the receiver —
  // stopped (an error), or its inbound filter — when the message arrives (:49-75; k_sync_delay)
  const bool loss = lost_k(c, out_loss(c, v, to), v, SWIM_STREAM_SYNC_OUT, ordinal, 0);
  const uint32_t k = !loss && c.delay_on ? delay_ticks(c, v, to, v, SWIM_STREAM_SYNC_DELAY, ordinal, 0) : 0u;
  if (!k && (loss || !c.up[to])) {
    if (initial) m.init_done++;
    return;
  }
  q.flags |= RQ_DELIVERED;
  if (k) { park_request(c, b, q, k); return; }
  if (!in_pass(c, to, v)) return;  // inbound-blocked at the receiver: silently dropped
  sflag_set(c, b, v - c.lo, owned(c, to) ? SF_SENT | SF_SENT_LOCAL : SF_SENT);
  if (!owned(c, to)) {  // content (this row) travels with the request: k_pack_rows
    const uint32_t d = owner(c, to);
    const uint32_t i = atomicAdd(&b.x->req[d], 1u);
    if (i >= b.tx_req_cap) { set_err(c, ERR_REQS); return; }
    b.tx_reqs[(size_t)d * b.tx_req_cap + i] = q;
    return;
  }
  enqueue_sync(c, b, 0, q, true);
}

// doSync (:339-357), FD-triggered SYNCs (:427-442) and start0's initial SYNC to every seed (:250-291)
// (sn, fl: the member's sync_next and mflag words, loaded by the caller)
// The common case, a periodic doSync and nothing else, with no per-link settings, partition or
// address routing: selectSyncAddress's first draw almost always names a member, so everything the
// SYNC needs — the candidate's membership and seed words, the sender's up / table size / loss, the
// candidate's up / inbound filter and both members' sflag words — is loaded in ONE batch before any
// decision, and the item / inbox counters are taken together: the collection costs a few dependent
// round trips instead of a dozen.  Same draws, same decisions, same results as the general path
// (when the first draw does not name a member, select_sync_address takes over from scratch).
__device__ inline unsigned long long sync_collect_fast(const Ctx& c, const Bufs& b, uint32_t v) {
  const uint32_t i = v - c.lo, t32 = (uint32_t)c.T;
  c.sync_next[i] = t32 + c.S;
  const uint32_t x0 = next_int(draw(c, v, SWIM_STREAM_SYNC_SELECT, 0, 0), c.n);
  MemberDev& m = mem(c, v);
  // ---- one batch of independent loads
  const uint8_t upv = c.up[v], upx = c.up[x0], seedx = c.is_seed[x0], inbx = c.default_inbound[x0];
  const uint8_t lossv = c.default_loss[v];
  const uint32_t ax = aux_row(c, v)[x0], tsz = m.table_size;
  const uint32_t sfv = b.sflag[i];
  const bool x_local = owned(c, x0);
  const uint32_t sfx = x_local ? b.sflag[x0 - c.lo] : 0u;
  if (!upv) return 0;  // (fd_sync_cnt is already 0: no MF_FDSYNC)
  uint32_t t = x0;
  if (!(x0 != v && ((ax & A_IN_MEMBERS) || seedx))) {
    t = select_sync_address(c, v);
    if (t == NONE) return 0;
  }
  SyncReq q;
  q.from = v; q.to = t; q.ordinal = 0; q.slot = 0;
  q.flags = tsz << RQ_RECS_SHIFT;
  q.content = NONE; q.snap = NONE; q.pad = 0;
  const bool up_t = t == x0 ? upx != 0 : c.up[t] != 0;
  if (!up_t || lost_k(c, lossv, v, SWIM_STREAM_SYNC_OUT, 0, 0)) return 1;  // tryFailOutbound
  if (!(t == x0 ? inbx : c.default_inbound[t])) return 1;                   // inbound-blocked: dropped
  q.flags |= RQ_DELIVERED;
  const bool local = owned(c, t);
  if (!local) {  // content (this row) travels with the request: k_pack_rows
    sflag_set_from(c, b, i, SF_SENT, sfv);
    const uint32_t d = owner(c, t);
    const uint32_t k = atomicAdd(&b.x->req[d], 1u);
    if (k >= b.tx_req_cap) { set_err(c, ERR_REQS); return 1; }
    b.tx_reqs[(size_t)d * b.tx_req_cap + k] = q;
    return 1;
  }
  // (the sender's SF_SENT | SF_SENT_LOCAL is set inside, its CAS beside the enqueue's atomics)
  enqueue_sync(c, b, 0, q, true, t == x0 ? sfx : b.sflag[t - c.lo], SF_SENT | SF_SENT_LOCAL, sfv);
  return 1;
}

// PAcks whose Monos have all completed (collection of tick T, member v up): a deferred SYNC_ACK is
// sent now (onSync's doOnSuccess, MembershipProtocolImpl.java:399-413) — a phantom SYNC at the front of
// v's inbox, whose SYNC_ACK this sub-phase sends with v's table after its SYNC merges; a start0 group
// leaves the count its doFinally waits for.  The ack's receiver is marked SF_SENT | SF_MULTI (merged
// into in the SYNC_ACK sub-phase; no lone-SYNC_ACK shortcut for another ack it gets), on another
// shard through an E2 marker.  Oracle: phase_sync's collection.
__device__ inline void pack_inject(const Ctx& c, const Bufs& b, uint32_t v) {
  const uint32_t i = v - c.lo, n = min(c.pa_n[i], c.pa_cap), t32 = (uint32_t)c.T;
  PAck* L = c.pa + (size_t)i * c.pa_cap;
  MemberDev& m = mem(c, v);
  uint32_t w = 0;
  for (uint32_t k = 0; k < n; ++k) {
    const PAck a = L[k];
    if (a.wn || a.gp || a.ready > t32) {
      if (w != k) L[w] = a;
      ++w;
      continue;
    }
    if (a.flags & PA_INIT) {
      m.init_pend--;
      continue;
    }
    SyncReq q;
    q.from = a.to; q.to = v; q.ordinal = 0; q.slot = 0;
    q.flags = RQ_PHANTOM | RQ_DELIVERED | ((a.flags & PA_INITIAL_ACK) ? RQ_INITIAL : 0u);
    q.content = NONE; q.snap = NONE; q.pad = a.seq;
    if (owned(c, a.to)) {
      sflag_set(c, b, a.to - c.lo, SF_SENT | SF_MULTI);
    } else {
      SyncReq mk = q;
      mk.from = v; mk.to = a.to; mk.flags = RQ_PHANTOM | RQ_DEFER;
      const uint32_t d = owner(c, a.to);
      const uint32_t j = atomicAdd(&b.x->req[d], 1u);
      if (j < b.tx_req_cap) b.tx_reqs[(size_t)d * b.tx_req_cap + j] = mk; else set_err(c, ERR_REQS);
    }
    enqueue_sync(c, b, 0, q, true);
  }
  c.pa_n[i] = w;
  if (w == 0) c.mflag[i] &= ~MF_PACK;
}

__device__ inline unsigned long long sync_collect_pre(const Ctx& c, const Bufs& b, uint32_t v, uint32_t sn, uint32_t fl) {
  const uint32_t i = v - c.lo, t32 = (uint32_t)c.T;
  const bool due = sn == t32;  // the periodic doSync timer fires (sync_on, phase sync_start)
  if (!due && !(fl & (MF_FDSYNC | MF_JOIN | MF_PACK))) return 0;
  if (due && !(fl & (MF_FDSYNC | MF_JOIN | MF_PACK)) && !c.n_links && !c.partition && !c.route && !c.delay_on &&
      !own_seeds(c, v))
    return sync_collect_fast(c, b, v);
  if (due) c.sync_next[i] = t32 + c.S;
  if (fl & MF_FDSYNC) c.mflag[i] = fl & ~MF_FDSYNC;
  MemberDev& m = mem(c, v);
  if (!c.up[v]) {
    m.fd_sync_cnt = 0;
    if (fl & MF_PACK) {  // a stopped member's waits and deferred acks are void
      c.pa_n[i] = 0;
      m.init_pend = 0;
      c.mflag[i] &= ~MF_PACK;
    }
    return 0;
  }
  uint32_t k = 0;
  unsigned long long nsync = 0;
  if (due) {
    uint32_t t = select_sync_address(c, v);
    if (t != NONE) { add_req(c, b, v, dst(c, t), k++, false); nsync++; }
  }
  for (uint32_t i = 0; i < m.fd_sync_cnt; ++i) {
    add_req(c, b, v, dst(c, c.fd_sync[(size_t)(v - c.lo) * FD_SYNC_MAX + i]), k++, false);
    nsync++;
  }
  m.fd_sync_cnt = 0;
  if (m.join_now) {
    m.init_total = 0;
    m.init_done = 0;
    uint32_t ns = 0;
    const uint32_t* sl = seeds_of(c, v, ns);
    for (uint32_t i = 0; i < ns; ++i) {
      uint32_t s = sl[i];
      if (s != v && dst(c, s) != v) { add_req(c, b, v, dst(c, s), k++, true); nsync++; }
    }
  }
  if (k > 1) sflag_set(c, b, i, SF_MULTI);  // (k_sync_apply's lone-SYNC_ACK shortcut needs k = 1)
  if (fl & MF_PACK) pack_inject(c, b, v);
  return nsync;
}
__device__ inline unsigned long long sync_collect_member(const Ctx& c, const Bufs& b, uint32_t v) {
  return sync_collect_pre(c, b, v, c.sync_next[v - c.lo], c.mflag[v - c.lo]);
}


#include "swim_sync.h"
#include "swim_quiet.h"


// ------------------------------------------------------------------------------- end of tick
// Boyer-Moore majority merge of two (candidate, count) pairs
__device__ __forceinline__ void bm_merge(uint32_t& c1, uint32_t& n1, uint32_t c2, uint32_t n2) {
  if (c1 == c2) n1 += n2;
  else if (n1 >= n2) n1 -= n2;
  else { c1 = c2; n1 = n2 - n1; }
}

// Rebase of the block witness (every kRebaseEvery ticks, inside k_end_tick, when no other kernel
// runs): for each subject whose record changed in some row since the last rebase, ref moves to the
// majority record of the live owned rows when that record is held by more live rows than the current
// ref, and every owned row's block count follows exactly (one pass over the column).  Any ref keeps
// bdiff exact; the majority only keeps it mostly zero.  Every thread of the grid calls it.
constexpr int REB_BLOCK = 256;
__device__ void rebase_witness(const Ctx& c) {
  __shared__ uint32_t s_list[REB_BLOCK], s_n;
  __shared__ uint32_t s_c[REB_BLOCK / 64], s_k[REB_BLOCK / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (uint32_t s0 = blockIdx.x * REB_BLOCK; s0 < c.n; s0 += gridDim.x * REB_BLOCK) {
    if (tid == 0) s_n = 0;
    __syncthreads();
    const uint32_t sj = s0 + tid;
    if (sj < c.n && c.dirty[sj]) {
      c.dirty[sj] = 0u;
      s_list[atomicAdd(&s_n, 1u)] = sj;
    }
    __syncthreads();
    const uint32_t ns = s_n;
    for (uint32_t q = 0; q < ns; ++q) {
      const uint32_t s = s_list[q];
      const uint32_t rf = c.ref[s];
      const uint32_t* col = c.recs + s;
      // pass 1: majority candidate of the live rows
      uint32_t cand = 0, cnt = 0;
      for (uint32_t v = tid; v < c.nl; v += REB_BLOCK)
        if (c.up[c.lo + v]) bm_merge(cand, cnt, col[(size_t)v * c.n], 1u);
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) {
        const uint32_t c2 = __shfl_xor(cand, d, 64), n2 = __shfl_xor(cnt, d, 64);
        bm_merge(cand, cnt, c2, n2);
      }
      if (lane == 0) { s_c[wv] = cand; s_k[wv] = cnt; }
      __syncthreads();
      cand = s_c[0];
      cnt = s_k[0];
      for (int w = 1; w < REB_BLOCK / 64; ++w) bm_merge(cand, cnt, s_c[w], s_k[w]);
      __syncthreads();
      // pass 2: live rows holding the candidate vs holding ref
      uint32_t hc = 0, hr = 0;
      if (cand != rf)
        for (uint32_t v = tid; v < c.nl; v += REB_BLOCK)
          if (c.up[c.lo + v]) {
            const uint32_t x = col[(size_t)v * c.n];
            hc += x == cand ? 1u : 0u;
            hr += x == rf ? 1u : 0u;
          }
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) {
        hc += __shfl_xor(hc, d, 64);
        hr += __shfl_xor(hr, d, 64);
      }
      if (lane == 0) { s_c[wv] = hc; s_k[wv] = hr; }
      __syncthreads();
      hc = hr = 0;
      for (int w = 0; w < REB_BLOCK / 64; ++w) { hc += s_c[w]; hr += s_k[w]; }
      __syncthreads();
      if (cand != rf && hc > hr) {
        // pass 3: every owned row's count of the subject's block follows the new ref
        const uint32_t blk = s >> BLK_SHIFT;
        for (uint32_t v = tid; v < c.nl; v += REB_BLOCK) {
          const uint32_t x = col[(size_t)v * c.n];
          const int d = (x != cand ? 1 : 0) - (x != rf ? 1 : 0);
          if (d) bdiff_add(c, v, blk, d);
        }
        if (tid == 0) c.ref[s] = cand;
      }
      __syncthreads();
    }
  }
}

// start0's doFinally (:285-289) for members that joined this tick; graceful leaves complete.
// ---- FETCH phase (message delay only): the delayed GET_METADATA legs arriving this tick, thread per
// owned viewer walking its chain of the previous tick's queue in issue order — a leg not due yet or a
// response now in flight moves to this tick's queue, a completed round trip is the fetch's doOnSuccess
// (apply_alive, events of SWIM_PHASE_FETCH) — then the workgroup applies the pingMembers inserts of its
// viewers.  A stopped viewer's round trips are void.  Oracle: phase_fetch.
__global__ void __launch_bounds__(256) k_fetch_due(KP) {
  const Ctx c = pctx(P, T);
  __shared__ uint32_t s_iP[256], s_iS[256], s_iR[256], s_list[256], s_n;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  if (i < c.nl) {
    const uint32_t pn = (uint32_t)T & 1u, po = pn ^ 1u;
    uint32_t cur = c.fq_head[(size_t)po * c.nl + i];
    c.fq_head[(size_t)pn * c.nl + i] = NONE;
    const uint32_t v = c.lo + i;
    if (cur != NONE && c.up[v]) {
      const FetchEnt* q = c.fq + (size_t)po * c.fq_cap;
      mem(c, v).ev_minor = 0;
      for (uint32_t guard = 0; cur != NONE && guard < c.fq_cap; ++guard) {
        if (cur >= c.fq_cap) { set_err(c, ERR_FETCHQ); break; }
        FetchEnt e = q[cur];
        cur = e.next;
        if (e.due > (uint32_t)T) {
          fq_push(c, v, e);
          continue;
        }
        const int r = (e.info >> 8) == 1u ? fetch_stage1(c, v, e) : (in_pass(c, v, e.d) ? 1 : 0);
        if (r == 2) {
          fq_push(c, v, e);
          continue;
        }
        if (e.link != NONE) {  // the Mono waiting on it ends now (a response) or at the timeout
          PAck* pa = pack_find(c, v, e.link);
          if (!pa) continue;  // cancelled with start0's Flux: its doOnSuccess never runs
          pa->wn--;
          pa->ready = max(pa->ready, r == 1 ? (uint32_t)T : e.t0 + mt_ticks(c));
        }
        if (r == 1) {
          stat_add(c, ST_FETCH_OK, 1);
          apply_alive(c, v, e.s, e.inc, (int)((e.info >> 4) & 15u), SWIM_PHASE_FETCH, e.ver);
        }
      }
      if (mem(c, v).ins_rank) s_list[atomicAdd(&s_n, 1u)] = v;
    }
  }
  __syncthreads();
  const uint32_t nv = s_n;
  for (uint32_t k = 0; k < nv; ++k) apply_ins_batch<256, true>(c, s_list[k], threadIdx.x, s_iP, s_iS, s_iR);
}

__global__ void __launch_bounds__(REB_BLOCK) k_end_tick(KP, int rebase) {
  const Ctx c = pctx(P, T);
  Counters* k = P->b.k;
  Xc* x = P->c.xchg ? P->b.x : nullptr;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (rebase) rebase_witness(c);
  {  // this tick's content snapshots are released; the next tick's slot counter starts at zero
    const Bufs& b = P->b;
    const uint32_t par = (uint32_t)(T & 1);
    const uint32_t ns = min(b.snap_cnt[par], b.snap_cap);
    for (uint32_t q = i; q < ns; q += gridDim.x * blockDim.x) {
      const uint32_t m = b.snap_list[par * b.snap_cap + q];
      b.snap_idx[m] = NONE;
      b.ack_snap[m] = NONE;
    }
    if (i == 0) b.snap_cnt[par ^ 1u] = 0;
    if (i == 0 && c.delay_on) b.dq_cnt[(uint32_t)T & DQ_MASK] = 0;  // this tick's delayed arrivals are delivered
    // the metadata queue read by this tick's FETCH phase is written next during tick T + 1
    if (i == 0 && c.fq) c.fq_cnt[((uint32_t)T & 1u) ^ 1u] = 0;
  }
  // collector blocks freed this tick become allocatable: tier t by workgroup t (the counters are
  // read, then rewritten, by the same threads), all tiers by workgroup 0 in a grid of fewer than 5
  for (int t = 0; t < NTIER; ++t) {
    if (blockIdx.x != (gridDim.x > NTIER ? (uint32_t)t : 0u)) continue;
    const int32_t a0 = c.spill_ctl[t].avail;
    const uint32_t a = a0 > 0 ? (uint32_t)a0 : 0u, f = min(c.spill_ctl[t].freed, c.spill_cap[t] - a);
    for (uint32_t j = threadIdx.x; j < f; j += blockDim.x) c.spill_avail[t][a + j] = c.spill_freed[t][j];
    __syncthreads();
    if (threadIdx.x == 0) {
      c.spill_ctl[t].avail = (int32_t)(a + f);
      c.spill_ctl[t].freed = 0;
    }
  }
  // timer-wheel pages freed this tick become allocatable (workgroup NTIER, as above)
  if (blockIdx.x == (gridDim.x > NTIER ? (uint32_t)NTIER : 0u)) {
    const int32_t a0 = c.wheel_ctl->avail;
    const uint32_t a = a0 > 0 ? (uint32_t)a0 : 0u, f = min(c.wheel_ctl->freed, c.wheel_pages - a);
    for (uint32_t j = threadIdx.x; j < f; j += blockDim.x) c.wheel_avail[a + j] = c.wheel_freed[j];
    __syncthreads();
    if (threadIdx.x == 0) {
      c.wheel_ctl->avail = (int32_t)(a + f);
      c.wheel_ctl->freed = 0;
    }
  }
  // park slots of the delayed SYNCs / SYNC_ACKs delivered this tick become allocatable (workgroup
  // NTIER + 1, as above)
  if (c.delay_on && blockIdx.x == (gridDim.x > NTIER + 1 ? (uint32_t)NTIER + 1 : 0u)) {
    const Bufs& b = P->b;
    const int32_t a0 = b.park_ctl->avail;
    const uint32_t a = a0 > 0 ? (uint32_t)a0 : 0u, f = min(b.park_ctl->freed, b.park_cap - a);
    for (uint32_t j = threadIdx.x; j < f; j += blockDim.x) b.park_avail[a + j] = b.park_freed[j];
    __syncthreads();
    if (threadIdx.x == 0) {
      b.park_ctl->avail = (int32_t)(a + f);
      b.park_ctl->freed = 0;
      b.sdq_cnt[(uint32_t)T & DQ_MASK] = 0;  // this tick's delayed SYNC arrivals are in the inboxes
    }
  }
  // receipt-bitmap slots requested this tick change owner (no other kernel runs now): their bit
  // cleared in every receiver's row, valid from the next tick; the other parity's queue (next tick's)
  // is emptied.  The claimed bits are gathered per row word in LDS first, so each row is touched once
  // per claimed word (a few words: claims come with new gossips)
  {
    const uint32_t par = (uint32_t)(T & 1);
    const uint32_t nclaim = min(c.gclaim_cnt[par], GSLOTS);  // (grid-uniform: nothing writes it now)
    if (nclaim) {
      __shared__ uint32_t s_cm[GROW], s_nz[GROW], s_nnz;
      for (uint32_t w = threadIdx.x; w < GROW; w += blockDim.x) s_cm[w] = 0;
      if (threadIdx.x == 0) s_nnz = 0;
      __syncthreads();
      for (uint32_t q = threadIdx.x; q < nclaim; q += blockDim.x) {
        const uint32_t e = c.gclaim[par * GSLOTS + q];
        if (e >> 31) atomicOr(&s_cm[(e & 0x7fffffffu) >> 5], 1u << (e & 31));  // (a first owner: nothing to clear)
      }
      __syncthreads();
      for (uint32_t w = threadIdx.x; w < GROW; w += blockDim.x)
        if (s_cm[w]) s_nz[atomicAdd(&s_nnz, 1u)] = w;
      __syncthreads();
      if (i < c.nl) {
        uint32_t* row = c.gbits + (size_t)i * GROW;
        const uint32_t nnz = s_nnz;
        for (uint32_t k2 = 0; k2 < nnz; ++k2) {
          const uint32_t w = s_nz[k2];
          row[w] &= ~s_cm[w];
        }
      }
      for (uint32_t q = i; q < nclaim; q += gridDim.x * blockDim.x) {
        const uint32_t sl = c.gclaim[par * GSLOTS + q] & 0x7fffffffu;
        c.gslot[sl].key = c.gpend[sl];
        c.gslot[sl].tick = (uint32_t)T + 1;
        c.gpend[sl] = 0;
      }
    }
    if (i == 0) c.gclaim_cnt[par ^ 1u] = 0;
  }
  // every other kernel of the tick has completed: reset the per-tick scratch counters
  if (i < sizeof(Counters) / 4) reinterpret_cast<uint32_t*>(k)[i] = 0;
  if (x && i < sizeof(Xc) / 4) reinterpret_cast<uint32_t*>(x)[i] = 0;
  if (x) {  // graceful leaves completed on other shards (k_recv_msgs took them)
    const uint32_t ns = *P->b.rx_stop_n;
    for (uint32_t q = i; q < ns; q += gridDim.x * blockDim.x) c.up[P->b.rx_stops[q]] = 0;
  }
  if (i >= c.nl) return;
  uint32_t fl = c.mflag[i];
  if (!(fl & (MF_JOIN | MF_LEAVE))) return;
  const uint32_t v = c.lo + i;
  MemberDev& m = c.mem[i];
  uint32_t keep = 0;
  // start0's doFinally (:285-289).  Every initial SYNC answered or failed fast: Flux.take completes,
  // and doFinally runs once the flatMap's inner Monos (the initial merges' fetches and LEAVING
  // spreads: PAck groups PA_INIT) have completed — periodic sync starts at the tick the last ended.
  // Else Flux.timeout (:281, restarted at every answer) fires at tick init_last + syncTimeout, cancels
  // the inner Monos still running (their fetches complete into nothing) and doFinally runs then.
  // MF_JOIN is kept while undecided.  Oracle: finish_joins.
  if (m.init_wait) {
    const uint64_t last = m.init_last;
    int64_t start = -1;
    if (m.init_done == m.init_total) {
      if (m.init_pend == 0) start = (int64_t)c.T;
    } else if (c.T + 1 >= last + c.sync_to_ticks) {
      start = (int64_t)(last + c.sync_to_ticks);
      if (m.init_pend) {  // the start0 groups are cancelled
        PAck* L = c.pa + (size_t)i * c.pa_cap;
        const uint32_t n = min(c.pa_n[i], c.pa_cap);
        uint32_t w = 0;
        for (uint32_t k = 0; k < n; ++k)
          if (!(L[k].flags & PA_INIT)) L[w++] = L[k];
        c.pa_n[i] = w;
        m.init_pend = 0;
        if (w == 0) fl &= ~MF_PACK;
      }
    }
    if (start >= 0) {
      m.sync_on = 1;
      m.sync_start = start;
      m.init_wait = 0;
      c.sync_next[i] = next_due(m.sync_start, c.T, c.S);
    } else {
      keep = MF_JOIN;
    }
  }
  m.join_now = 0;
  c.mflag[i] = (fl & ~(MF_JOIN | MF_LEAVE)) | keep;
  if (m.leave_done) {
    m.leave_done = 0;
    m.leave_pending = 0;
    c.up[v] = 0;
  }
}

// ------------------------------------------------------------------------------- KAT kernels
__global__ void k_kat_overrides(const int32_t* cases, uint32_t n, uint8_t* out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t* k = cases + 5 * i;
  out[i] = is_overrides((uint32_t)k[0], k[1], k[2] != 0, (uint32_t)k[3], k[4]) ? 1 : 0;
}

// SequenceIdCollectorTest through the engine's own collector code (inline entry + spill tiers)
__global__ void k_kat_collector(Ctx c, const uint8_t* kinds, const int64_t* values, uint32_t n, int64_t* res,
                                CollEnt* e) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  e->key = 1; e->lo = e->hi = 0; e->meta = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t x = (uint32_t)values[i];
    switch (kinds[i]) {
      case 0: res[i] = coll_add(c, e, x) ? 1 : 0; break;
      case 1: res[i] = coll_contains(c, e, x) ? 1 : 0; break;
      case 2: res[i] = coll_size(c, e); break;
      default: coll_clear(c, e); res[i] = 0; break;
    }
  }
}

__global__ void k_kat_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) philox4(ctr, key[0], key[1], out);
}

}  // namespace swimdev
