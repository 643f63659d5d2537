// swim_kernels.h — the HIP kernels of one lockstep tick.
//
// Phase A  k_fd (per 256-viewer block)                suspicion timeouts
// Phase B  k_fd                                       list compaction after REMOVED, then ping /
//                                                     ping-req / ack resolution + FD events
// Phase C  round start (+ segmentation) in k_fd, k_gossip_emit, k_alloc, k_scatter_msgs, k_gossip_deliver
// Phase D  SYNC collection (in k_fd / k_gossip_deliver), k_sync_prep, k_sync_classify, k_sync_apply (swim_sync.h; SYNC and SYNC_ACK)
// lists    (k_gossip_deliver, k_sync_apply)           deferred pingMembers inserts of ADDED events
// tick end k_end_tick
//
// Every kernel reads its work size from device memory (grid-stride over device counters), so the
// host never synchronises inside a tick.
#pragma once
#include "swim_device.h"

namespace swimdev {

// per-tick scratch counters, zeroed by one hipMemsetAsync at the start of every tick
struct Counters {
  uint32_t msg_total, msg_cursor, pad0;
  uint32_t req_total, req_recv_cnt, req_cursor;
  uint32_t ack_total, ack_recv_cnt, ack_cursor;
  uint32_t ins_total, ins_list_cnt;    // list inserts of the gossip phase
  uint32_t ins_total2, ins_list_cnt2;  // list inserts of the SYNC phase
  uint32_t pool_cursor;  // complex-record pool of the SYNC classify kernel
  uint32_t sender_cnt;   // senders of this tick's gossip round with live gossips
  uint32_t pad[2];
};

// per-tick message counts by destination shard (sharded engines), zeroed by k_end_tick
constexpr int MAXW = 16;
struct Xc {
  uint32_t msg[MAXW], req[MAXW], ack[MAXW];
  uint32_t stop;
  uint32_t pad[3];
};

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
  const GMsgFull* rx_msgs;
  const SyncReq* rx_reqs;
  const uint32_t* rx_rows;  // record rows of received SYNC / SYNC_ACKs, indexed by SyncReq.content
  const uint32_t* rx_stops;
  GMsgFull* msgs;      // produced in emit order
  GMsgFull* msgs_out;  // grouped by receiver
  uint32_t msg_cap;
  uint32_t* msg_cnt;   // per receiver
  uint32_t* msg_start;
  SyncReq* reqs;
  SyncReq* reqs_out;
  uint32_t req_cap;
  uint32_t* req_cnt;
  uint32_t* req_start;
  uint32_t* req_recv;
  uint2* req_desc;  // per receiver-list position: (inbox start, message count), written by k_sync_prep
  SyncReq* acks;
  SyncReq* acks_out;
  uint32_t* ack_cnt;
  uint32_t* ack_start;
  uint32_t* ack_recv;
  uint2* ack_desc;
  uint32_t* snap;       // snapshot record rows
  uint32_t snap_cap;
  uint32_t* snap_idx;   // per member: slot or NONE
  uint32_t* snap_list;
  uint32_t* snap_cnt;   // claims made by the last k_sync_prep (persistent across ticks)
  uint64_t* pend;       // per sync-apply workgroup: pending ALIVE admissions
  uint2* item_chunk;    // per (message, chunk): (pool base, complex count)
  uint32_t* item_total; // per message: complex count over all chunks
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
  for (uint32_t v = c.lo + blockIdx.x; v < c.lo + c.nl; v += gridDim.x) {
    uint32_t* r = rec_row(c, v);
    uint32_t* a = aux_row(c, v);
    const bool init = v < n_initial;
    for (uint32_t s = threadIdx.x; s < c.n; s += blockDim.x) {
      const bool in = init && s < n_initial;
      r[s] = in ? REC_IN_TABLE : 0u;  // ALIVE, incarnation 0
      a[s] = in ? (s == v ? A_IN_MEMBERS : conv_aux) : 0u;
    }
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
  m.fd_start = (int64_t)c.T;
  m.g_start = (int64_t)c.T;
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
  const uint32_t qcap = c.wheel_cap / c.wheel_nq;
  uint32_t* qc = c.wheel_cnt + (size_t)bucket * c.wheel_nq + blockIdx.x;
  const uint32_t cnt = min(*qc, qcap);
  const uint64_t* ent = c.wheel + (size_t)bucket * c.wheel_cap + (size_t)blockIdx.x * qcap;
  const uint32_t tmask = (uint32_t)(c.T & SWIM_DEADLINE_MASK);
  unsigned long long fired = 0;
  for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
    uint64_t e = ent[i];
    uint32_t v = (uint32_t)(e >> 32), s = (uint32_t)e;
    if (!c.up[v]) continue;
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
  if (threadIdx.x == 0 && cnt) *qc = 0;
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
// id, so the first relayed ack to reach the issuer completes every pending relay request.
__device__ inline void ping_req(const Ctx& c, uint32_t v, uint32_t t, unsigned long long& nev,
                                unsigned long long& nreq) {
  uint32_t relays[16];
  uint32_t nr = select_relays(c, v, t, relays);
  if (nr == 0) { publish_fd(c, v, t, SWIM_SUSPECT, nev); return; }
  nreq++;
  uint32_t pending_mask = 0, npend = 0;
  for (uint32_t j = 0; j < nr; ++j) {
    if (out_fail(c, v, relays[j], v, SWIM_STREAM_PINGREQ_OUT, j, 0)) publish_fd(c, v, t, SWIM_SUSPECT, nev);
    else { pending_mask |= 1u << j; npend++; }
  }
  if (npend == 0) return;
  int32_t arrived = -1;
  for (uint32_t j = 0; j < nr; ++j) {
    if (!(pending_mask & (1u << j))) continue;
    uint32_t r = relays[j];
    if (in_pass(c, r, v) && !out_fail(c, r, t, v, SWIM_STREAM_TRANSIT_PING_OUT, j, 0) &&
        in_pass(c, t, r) && !out_fail(c, t, r, v, SWIM_STREAM_TRANSIT_ACK_OUT, j, 0) &&
        in_pass(c, r, t) && !out_fail(c, r, v, v, SWIM_STREAM_RELAY_ACK_OUT, j, 0)) {
      arrived = (int32_t)j;
      break;
    }
  }
  if (arrived >= 0 && in_pass(c, v, relays[arrived])) {
    for (uint32_t i = 0; i < npend; ++i) publish_fd(c, v, t, SWIM_ALIVE, nev);
  } else {
    MemberDev& m = mem(c, v);
    m.relay_due = c.T + c.relay_ticks;
    m.relay_target = t;
    m.relay_pending = npend;
  }
}

__device__ inline void fd_member(const Ctx& c, uint32_t v, unsigned long long& nev, unsigned long long& nreq,
                                 unsigned long long& npings) {
  MemberDev& m = mem(c, v);
  if (!c.up[v]) return;  // a stopped member's timers stop; a join restarts them (fd_next)
  const bool due = (int64_t)c.T > m.fd_start && ((int64_t)c.T - m.fd_start) % c.P == 0;
  c.fd_next[v - c.lo] = fd_next_of(c, m, c.T);  // ack / relay timeouts set below are > T
  if (!due && m.relay_due != c.T && m.ack_due != c.T) return;
  m.ev_minor = 0;
  if (m.relay_due == c.T) {  // relay timeouts (:200-209)
    uint32_t t = m.relay_target, k = m.relay_pending;
    m.relay_due = 0;
    for (uint32_t i = 0; i < k; ++i) publish_fd(c, v, t, SWIM_SUSPECT, nev);
  }
  if (m.ack_due == c.T) {  // pingTimeout elapsed
    uint32_t t = m.ack_target;
    m.ack_due = 0;
    ping_req(c, v, t, nev, nreq);
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
      if (out_fail(c, v, t, v, SWIM_STREAM_PING_OUT, 0, 0)) {
        ping_req(c, v, t, nev, nreq);
      } else if (in_pass(c, t, v) && !out_fail(c, t, v, v, SWIM_STREAM_ACK_OUT, 0, 0) && in_pass(c, v, t)) {
        publish_fd(c, v, t, SWIM_ALIVE, nev);
      } else {
        m.ack_due = c.T + c.to_ticks;
        m.ack_target = t;
      }
    }
  }
  c.fd_next[v - c.lo] = fd_next_of(c, m, c.T);
}

// ------------------------------------------------------------------------------- phase C
__device__ __forceinline__ bool gossip_due(const Ctx& c, uint32_t v, const MemberDev& m) {
  return c.up[v] && (int64_t)c.T > m.g_start && ((int64_t)c.T - m.g_start) % c.G == 0;
}

// checkGossipSegmentation (GossipProtocolImpl.java:217-236); only launched when the threshold is
// below the inline interval capacity (otherwise a clear can never trigger).

// a GOSSIP_REQ for a receiver owned by this shard joins the receiver's inbox
__device__ inline void deliver_local_msg(const Ctx& c, const Bufs& b, GMsgFull msg) {
  const uint32_t i = atomicAdd(&b.k->msg_total, 1u);
  if (i >= b.msg_cap) { set_err(c, ERR_MSGS); return; }
  msg.slot = atomicAdd(&b.msg_cnt[msg.to - c.lo], 1u);
  b.msgs[i] = msg;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// doSpreadGossip (:141-184), wave-parallel.  Each wave owns the senders wid, wid + nw, ... and
// first checks up to 64 of them at once (lane l: sender base + l * nw): every due sender advances
// its period (:143); a sender with live gossips then gets the whole wave: lane 0 selects the
// targets (:322-343), the (target, slab position) pairs of selectGossipsToSend (:311-320) are
// spread over the lanes — loss draws and receiver-collector probes of 64 pairs in flight together,
// one enqueue atomic per (target, pass) — then the order-preserving sweep and the futures.
constexpr int EMIT_WAVES = 4;
// message slots are reserved in per-wave chunks (cb, cl: chunk base / slots left, wave-uniform); a
// pass fills the chunk's remainder and continues in a fresh chunk, so only the wave's last
// remainder is left over, marked as holes (to = NONE) that k_scatter_msgs skips
constexpr uint32_t EMIT_CHUNK = 128;
__device__ inline void emit_mark_holes(const Bufs& b, uint32_t cb, uint32_t cl, uint32_t lane) {
  for (uint32_t i = lane; i < cl; i += 64)
    if (cb + i < b.msg_cap) b.msgs[cb + i].to = NONE;
}
__device__ inline unsigned long long gossip_emit_sender(const Ctx& c, const Bufs& b, uint32_t v, uint64_t period,
                                                        uint32_t glen, uint32_t lane, uint32_t* s_t, uint32_t& cb,
                                                        uint32_t& cl, unsigned long long& nmat) {
  MemberDev& m = mem(c, v);
  const uint32_t rlen = m.remote_len;
  const uint32_t F = (uint32_t)c.fanout;
  if (lane == 0) {  // selectGossipMembers (:322-343)
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
  }
  __syncwarp();
  const uint32_t nt = s_t[0];
  const uint64_t spread = (uint64_t)(c.repeat_mult * ceil_log2(rlen + 1));
  const uint64_t sweep = 2 * (spread + 1);
  GossipDev* slab = slab_of(c, v);
  unsigned long long nmsg = 0;
  // lane = slab position: one GossipState read serves all nt targets, whose loss draws and
  // receiver checks are independent (issued together); messages keep the (target, position) keys
  for (uint32_t p0 = 0; p0 < glen; p0 += 64) {
    const uint32_t p = p0 + lane;
    GossipDev g;
    bool win = false;
    if (p < glen) {
      g = slab[p];
      win = (uint64_t)g.inf_period + spread >= period;
    }
    uint32_t matb = 0;  // bit j: a message to target j is materialised
    if (__ballot(win)) {
      for (uint32_t j = 0; j < nt; ++j) {
        const uint32_t t = s_t[1 + j];
        const bool send = win && !gossip_infected(g, t);
        nmsg += send ? 1u : 0u;
        // delivered copies; a receiver on this shard that already holds the sequence id drops it
        // (its collector only grows until delivery), another shard filters on arrival
        const bool mat = send && c.up[t] && in_pass(c, t, v) &&
                         !lost_k(c, out_loss(c, v, t), v, SWIM_STREAM_GOSSIP_OUT, j, p) &&
                         !(owned(c, t) && known_received(c, t, g.gossiper, g.seq));
        matb |= (mat ? 1u : 0u) << j;
      }
    }
    if (!__ballot(matb != 0)) continue;
    // one enqueue per target present in this pass: lane j issues target j's receiver atomic; the
    // message slots of this shard's targets come out of the wave's chunk, in (target, lane) order
    uint32_t base = 0, slot = 0, cnt_mine = 0, loc_off = 0, loc_tot = 0;
    for (uint32_t j = 0; j < nt; ++j) {
      const uint32_t cj = (uint32_t)__popcll(__ballot((matb >> j) & 1u));
      nmat += cj;  // wave-uniform
      if (lane == j) cnt_mine = cj;
      if (owned(c, s_t[1 + j])) {
        if (lane == j) loc_off = loc_tot;
        loc_tot += cj;
      }
    }
    uint32_t nb = 0, want = 0;
    if (loc_tot > cl) {
      want = loc_tot - cl > EMIT_CHUNK ? loc_tot - cl : EMIT_CHUNK;
      if (lane == 0) nb = atomicAdd(&b.k->msg_total, want);
      nb = __shfl(nb, 0, 64);
    }
    if (lane < nt && cnt_mine) {
      const uint32_t tj = s_t[1 + lane];
      if (owned(c, tj)) {
        base = loc_off;  // index in this pass's local sequence; mapped to a slot below
        slot = atomicAdd(&b.msg_cnt[tj - c.lo], cnt_mine);
      } else {
        base = atomicAdd(&b.x->msg[owner(c, tj)], cnt_mine);
      }
    }
    for (uint32_t j = 0; j < nt; ++j) {
      const bool mat = (matb >> j) & 1u;
      const uint64_t mk = __ballot(mat);
      if (!mk) continue;
      const uint32_t bj = __shfl(base, (int)j, 64), sj = __shfl(slot, (int)j, 64);
      if (!mat) continue;
      const uint32_t pre = lanes_below(mk);
      const uint32_t t = s_t[1 + j];
      GMsgFull msg;
      msg.to = t; msg.from = v; msg.pos = p; msg.slot = sj + pre;
      msg.gossiper = g.gossiper; msg.seq = g.seq; msg.subject = g.subject; msg.status = g.status;
      msg.inc = g.inc; msg.pad[0] = msg.pad[1] = msg.pad[2] = 0;
      if (owned(c, t)) {
        const uint32_t seq_i = bj + pre;  // position in the pass's local sequence
        const uint32_t loc_slot = seq_i < cl ? cb + seq_i : nb + (seq_i - cl);
        if (loc_slot < b.msg_cap) b.msgs[loc_slot] = msg; else set_err(c, ERR_MSGS);
      } else {
        const uint32_t d = owner(c, t);
        if (bj + pre < b.tx_msg_cap) b.tx_msgs[(size_t)d * b.tx_msg_cap + bj + pre] = msg; else set_err(c, ERR_MSGS);
      }
    }
    if (loc_tot > cl) {
      cb = nb + (loc_tot - cl);
      cl = want - (loc_tot - cl);
    } else {
      cb += loc_tot;
      cl -= loc_tot;
    }
  }
  // sweep (:158-164, :350-358), order preserving: a chunk's survivors land at or below their own
  // positions, all of which the wave has already read
  uint32_t w = 0;
  bool done = false;
  const bool leaving = m.leave_pending != 0;
  for (uint32_t p0 = 0; p0 < glen; p0 += 64) {
    const uint32_t p = p0 + lane;
    GossipDev g;
    bool keep = false;
    if (p < glen) {
      g = slab[p];
      keep = !(period > (uint64_t)g.inf_period + sweep);
    }
    const uint64_t mask = __ballot(keep);
    if (keep) {
      slab[w + lanes_below(mask)] = g;
      // futures (:167-180): the graceful-leave future stops the member at the end of the tick
      if (leaving && period > (uint64_t)g.inf_period + spread && g.gossiper == m.leave_gossiper &&
          g.seq == (uint32_t)m.leave_seq)
        done = true;
    }
    w += (uint32_t)__popcll(mask);
  }
  const bool any_done = __ballot(done) != 0;
  if (lane == 0) {
    m.gossip_len = w;
    if (any_done) {
      m.leave_done = 1;
      c.mflag[v - c.lo] |= MF_LEAVE;
      if (c.world > 1) {  // every shard stops sending to v at the end of this tick
        const uint32_t i = atomicAdd(&b.x->stop, 1u);
        if (i < b.tx_stop_cap) b.tx_stops[i] = v; else set_err(c, ERR_MSGS);
      }
    }
  }
  __syncwarp();
  return nmsg;
}

// doSpreadGossip's first steps for a due sender (one thread each, run by k_fd right after the
// member's FD step: both touch only the member's own state): period++ (:143) and, when it holds live
// gossips (:149-151), a place in the round's sender list (called by every lane of a wave: the list
// append is one atomic per wave)
__device__ __forceinline__ void gossip_round(const Ctx& c, const Bufs& b, uint32_t i) {
  bool busy = false;
  if (i < c.nl) {
    MemberDev& m = c.mem[i];
    if (gossip_due(c, c.lo + i, m)) {
      const uint64_t period = m.g_period;
      m.g_period = period + 1;
      m.period_used = period;
      // checkGossipSegmentation (:217-236): clear collectors holding more than the threshold of
      // intervals; only viewers whose collector crossed it since their last round look
      if (c.seg_flag[i]) {
        c.seg_flag[i] = 0;
        CollEnt* base = c.coll + (size_t)i * c.hcap;
        for (uint32_t j = 0; j < c.hcap; ++j)
          if (base[j].key && (int32_t)coll_size(c, base + j) > c.seg_threshold) {
            coll_clear(c, base + j);
            c.clr_tick[i] = (uint32_t)c.T;
          }
      }
      busy = m.gossip_len != 0;  // else no target selection, no shuffle draw
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
__device__ inline unsigned long long sync_collect_member(const Ctx& c, const Bufs& b, uint32_t v);

// collect (ticks without a gossip round): the member's SYNC requests of phase D are collected here
// too, right after its FD step.  Nothing between k_fd and phase D on such a tick touches the state
// sync_collect_member reads (the member's own lists, schedule, fd_sync queue), so this equals the
// separate k_sync_collect launch and saves its round trips.
__global__ void __launch_bounds__(256) k_fd(KP, int gossip, int collect) {
  const Ctx c = pctx(P, T);
  __shared__ uint32_t s_list[256];
  __shared__ uint32_t s_cnt;
  timers_block(c, T);  // phase A for this block's viewers
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
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
  if (i < c.nl && c.fd_next[i] == (uint32_t)T) fd_member(c, c.lo + i, nev, nreq, npings);
  if (gossip) gossip_round(c, P->b, i);  // phase C's first step for this member
  if (collect) {
    const Ctx cs = pctx_sync(P, T);
    const unsigned long long nsync = i < c.nl ? sync_collect_member(cs, P->b, c.lo + i) : 0;
    wave_stat_add(cs, ST_SYNCS, nsync);
  }
  wave_stat_add(c, ST_FD_EVENTS, nev);
  wave_stat_add(c, ST_PING_REQS, nreq);
  wave_stat_add(c, ST_PINGS, npings);
}

// the rest of the round for the listed senders: one sender per wave at a time
// prof (sampled launches only): {GOSSIP_REQs materialised, (gossip, sender round) states read}
__global__ void __launch_bounds__(64 * EMIT_WAVES) k_gossip_emit(KP, unsigned long long* prof) {
  __shared__ uint32_t s_t[EMIT_WAVES][17];
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t ns = b.k->sender_cnt;
  unsigned long long nmsg = 0, nmat = 0, nstate = 0;
  uint32_t cb = 0, cl = 0;
  for (uint32_t k = __builtin_amdgcn_readfirstlane(blockIdx.x * EMIT_WAVES + wv); k < ns; k += gridDim.x * EMIT_WAVES) {
    const uint32_t i = b.senders[k];
    const MemberDev& m = c.mem[i];
    const uint32_t glen = m.gossip_len;
    nstate += glen;
    nmsg += gossip_emit_sender(c, b, c.lo + i, m.g_period - 1, glen, lane, s_t[wv], cb, cl, nmat);
  }
  emit_mark_holes(b, cb, cl, lane);
  if (prof && lane == 0 && nstate) {
    atomicAdd(prof, nmat);
    atomicAdd(prof + 1, nstate);
  }
  wave_stat_add(c, ST_GOSSIP_MESSAGES, nmsg);
}

// GOSSIP_REQs arriving from other shards: drop provable duplicates (the emitter could not see
// this shard's collectors), then join the local message list exactly as a local send does
__global__ void k_recv_msgs(KP, uint32_t nrx) {
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nrx; i += gridDim.x * blockDim.x) {
    const GMsgFull msg = b.rx_msgs[i];
    if (coll_contains(c, coll_find(c, msg.to, msg.gossiper), msg.seq)) continue;
    deliver_local_msg(c, b, msg);
  }
}

// group-by-receiver: region start per receiver (a workgroup scan of 256 receivers' counts and one
// cursor atomic per workgroup), then scatter by (start + arrival slot)
__global__ void __launch_bounds__(256) k_alloc(KP) {
  __shared__ uint32_t s_wave[256 / 64 + 1];
  __shared__ uint32_t s_base;
  const Bufs b = P->b;
  const uint32_t nl = P->c.nl;
  if (b.k->msg_total == 0) return;  // a round without messages (every msg_cnt is 0)
  for (uint32_t base = blockIdx.x * 256; base < nl; base += gridDim.x * 256) {
    const uint32_t r = base + threadIdx.x;
    const uint32_t k = r < nl ? b.msg_cnt[r] : 0u;
    uint32_t total;
    const uint32_t off = block_exclusive_scan<256>(k, s_wave, &total);
    if (threadIdx.x == 0) s_base = total ? atomicAdd(&b.k->msg_cursor, total) : 0u;
    __syncthreads();
    if (k) b.msg_start[r] = s_base + off;
    __syncthreads();
  }
}

__global__ void k_scatter_msgs(KP) {
  const Bufs b = P->b;
  const uint32_t lo = P->c.lo;
  const uint32_t n = min(b.k->msg_total, b.msg_cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const GMsgFull m = b.msgs[i];
    if (m.to == NONE) continue;  // a hole of a wave's slot chunk (k_gossip_emit)
    const uint64_t at = (uint64_t)b.msg_start[m.to - lo] + m.slot;
    if (at < b.msg_cap) b.msgs_out[at] = m;  // beyond: the buffer overflowed (ERR_MSGS is set)
  }
}

__device__ __forceinline__ uint64_t msg_key(const GMsgFull& m) { return ((uint64_t)m.from << 32) | m.pos; }

// heap sort of one receiver's messages by (sender, slab position)
__device__ inline void sort_msgs(GMsgFull* a, uint32_t n) {
  if (n < 2) return;
  if (n <= 16) {
    for (uint32_t i = 1; i < n; ++i) {
      GMsgFull x = a[i];
      uint64_t kx = msg_key(x);
      int32_t j = (int32_t)i - 1;
      while (j >= 0 && msg_key(a[j]) > kx) { a[j + 1] = a[j]; --j; }
      a[j + 1] = x;
    }
    return;
  }
  auto sift = [&](uint32_t start, uint32_t end) {
    uint32_t root = start;
    while (2 * root + 1 < end) {
      uint32_t ch = 2 * root + 1;
      if (ch + 1 < end && msg_key(a[ch]) < msg_key(a[ch + 1])) ch++;
      if (msg_key(a[root]) < msg_key(a[ch])) { GMsgFull t = a[root]; a[root] = a[ch]; a[ch] = t; root = ch; }
      else return;
    }
  };
  for (int64_t s = (int64_t)n / 2 - 1; s >= 0; --s) sift((uint32_t)s, n);
  for (uint32_t e = n - 1; e > 0; --e) {
    GMsgFull t = a[0]; a[0] = a[e]; a[e] = t;
    sift(0, e);
  }
}

// onGossipReq (GossipProtocolImpl.java:201-215) for one received message, in canonical order
__device__ inline bool on_gossip_req(const Ctx& c, uint32_t r, MemberDev& m, GossipDev* slab, const GMsgFull& g) {
  CollEnt* col = coll_ensure(c, r, g.gossiper);
  if (!col) return false;
  const bool was_cleared = (col->meta & COLL_CLEARED) != 0;
  if (!coll_add(c, col, g.seq, &c.seg_flag[r - c.lo])) return false;
  receipt_mark(c, r, g.gossiper, g.seq);
  int32_t found = -1;
  if (was_cleared) {  // a GossipState can outlive its collector entry only after a clear
    for (uint32_t p = 0; p < m.gossip_len; ++p)
      if (slab[p].gossiper == g.gossiper && slab[p].seq == g.seq) { found = (int32_t)p; break; }
  }
  if (found < 0) {
    if (m.gossip_len >= c.gcap) { set_err(c, ERR_SLAB); return true; }
    GossipDev ns;
    ns.gossiper = g.gossiper; ns.seq = g.seq; ns.subject = g.subject; ns.status = g.status; ns.inc = g.inc;
    ns.inf_period = (uint32_t)m.g_period;
    ns.inf[0] = g.from;
#pragma unroll
    for (int k = 1; k < GINF; ++k) ns.inf[k] = NONE;
    slab[m.gossip_len++] = ns;
    // onMembershipGossip (MembershipProtocolImpl.java:452-459)
    if (update_membership(c, r, g.subject, g.status, g.inc, R_GOSSIP, SWIM_PHASE_GOSSIP))
      apply_alive(c, r, g.subject, g.inc, R_GOSSIP, SWIM_PHASE_GOSSIP);
  } else {
    GossipDev& st = slab[found];
    if (!gossip_infected(st, g.from)) {
      int k = 0;
      while (k < GINF && st.inf[k] != NONE) ++k;
      if (k < GINF) st.inf[k] = g.from;
      else set_err(c, ERR_INFECTED);
    }
  }
  return true;
}

// One receiver per thread (the onGossipReq chain of a receiver is sequential, so concurrency comes
// from many receivers): the inbox keys (sender, slab position) are insertion-sorted in an LDS slice
// laid out [slot][thread] (conflict-free), then processed in that order.  Inboxes above DLV_SORT
// messages are deferred to the workgroup: one wave bitonic-sorts up to DLV_BIG keys in LDS and its
// lane 0 processes them; larger inboxes are sorted in place in global memory.
constexpr int DLV_BLOCK = 256;
#ifndef DLV_SORT_N
#define DLV_SORT_N 24
#endif
constexpr int DLV_SORT = DLV_SORT_N;
constexpr int DLV_BIG = 512;
__device__ inline unsigned long long deliver_sorted(const Ctx& c, uint32_t r, const GMsgFull* a, uint32_t k,
                                                    const uint8_t* ix8, uint32_t ix8_stride, const uint16_t* ix16) {
  MemberDev& m = mem(c, r);
  m.ev_minor = 0;
  m.fetch_ctr = 0;
  GossipDev* slab = slab_of(c, r);
  unsigned long long acc = 0;
  for (uint32_t q = 0; q < k; ++q) {
    const uint32_t at = ix8 ? ix8[q * ix8_stride] : ix16 ? ix16[q] : q;
    if (on_gossip_req(c, r, m, slab, a[at])) acc++;
  }
  return acc;
}

__device__ void apply_ins_chain(const Ctx& c, uint32_t v);
__device__ inline unsigned long long sync_collect_member(const Ctx& c, const Bufs& b, uint32_t v);

// phase D's SYNC collection for this workgroup's members (same member -> workgroup mapping as the
// delivery loop), after their deliveries and inserts: nothing else in the gossip phase touches what
// sync_collect_member reads (the member's own lists, schedule, fd_sync queue)
__device__ inline void deliver_collect(KP) {
  const Ctx cs = pctx_sync(P, T);
  unsigned long long nsync = 0;
  for (uint32_t base = blockIdx.x * DLV_BLOCK; base < cs.nl; base += gridDim.x * DLV_BLOCK) {
    const uint32_t i = base + threadIdx.x;
    if (i < cs.nl) nsync += sync_collect_member(cs, P->b, cs.lo + i);
  }
  wave_stat_add(cs, ST_SYNCS, nsync);
}

// Delivery, then the gossip phase's deferred pingMembers inserts of this workgroup's receivers: a
// viewer's ADDED events of the phase all come from the one thread that delivered to it (on_added),
// and no delivery reads another viewer's ping list, so a receiver's op chain is complete, and may be
// applied, as soon as its own workgroup has delivered (no separate k_ins_apply launch).  Then the
// members' SYNC collection (no separate k_sync_collect launch).
__global__ void __launch_bounds__(DLV_BLOCK) k_gossip_deliver(KP) {
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  __shared__ uint64_t s_key[DLV_SORT][DLV_BLOCK];
  __shared__ uint8_t s_ix[DLV_SORT][DLV_BLOCK];
  __shared__ uint64_t s_bkey[DLV_BLOCK / 64][DLV_BIG];
  __shared__ uint16_t s_bix[DLV_BLOCK / 64][DLV_BIG];
  __shared__ uint32_t s_big_r[DLV_BLOCK], s_big_k[DLV_BLOCK], s_big_start[DLV_BLOCK];
  __shared__ uint32_t s_nbig;
  if (b.k->msg_total == 0) {  // a round without messages: no receiver has an inbox
    deliver_collect(P, T);
    return;
  }
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_nbig = 0;
  __syncthreads();
  unsigned long long acc = 0;
  for (uint32_t i = blockIdx.x * DLV_BLOCK + tid; i < c.nl; i += gridDim.x * DLV_BLOCK) {
    const uint32_t k = b.msg_cnt[i];
    if (k == 0) continue;
    const uint32_t r = c.lo + i;
    const uint32_t start = b.msg_start[r - c.lo];
    b.msg_cnt[r - c.lo] = 0;
    if (!c.up[r]) continue;
    if ((uint64_t)start + k > b.msg_cap) {  // the message buffer overflowed (ERR_MSGS already set)
      set_err(c, ERR_MSGS);
      continue;
    }
    GMsgFull* a = b.msgs_out + start;
    if (k <= (uint32_t)DLV_SORT) {
      for (uint32_t q = 0; q < k; ++q) {
        const uint64_t kx = ((uint64_t)a[q].from << 32) | a[q].pos;  // keys are unique
        int32_t j = (int32_t)q - 1;
        while (j >= 0 && s_key[j][tid] > kx) {
          s_key[j + 1][tid] = s_key[j][tid];
          s_ix[j + 1][tid] = s_ix[j][tid];
          --j;
        }
        s_key[j + 1][tid] = kx;
        s_ix[j + 1][tid] = (uint8_t)q;
      }
      acc += deliver_sorted(c, r, a, k, &s_ix[0][tid], DLV_BLOCK, nullptr);
      continue;
    }
    if (k <= (uint32_t)DLV_BIG) {
      const uint32_t slot = atomicAdd(&s_nbig, 1u);
      if (slot < DLV_BLOCK) {
        s_big_r[slot] = r;
        s_big_k[slot] = k;
        s_big_start[slot] = start;
        continue;
      }
    }
    sort_msgs(a, k);
    acc += deliver_sorted(c, r, a, k, nullptr, 0, nullptr);
  }
  __syncthreads();
  const uint32_t nbig = min(s_nbig, (uint32_t)DLV_BLOCK);
  uint64_t* key = s_bkey[wv];
  uint16_t* ix = s_bix[wv];
  for (uint32_t bi = wv; bi < nbig; bi += DLV_BLOCK / 64) {
    const uint32_t r = s_big_r[bi], k = s_big_k[bi];
    const GMsgFull* a = b.msgs_out + s_big_start[bi];
    uint32_t P = 64;
    while (P < k) P <<= 1;
    for (uint32_t q = lane; q < P; q += 64) {
      key[q] = q < k ? (((uint64_t)a[q].from << 32) | a[q].pos) : ~0ull;
      ix[q] = (uint16_t)q;
    }
    __syncwarp();
    for (uint32_t size = 2; size <= P; size <<= 1)
      for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
        for (uint32_t t = lane; t < P / 2; t += 64) {
          const uint32_t lo = 2 * stride * (t / stride) + (t % stride), hi = lo + stride;
          const bool asc = (lo & size) == 0;
          const uint64_t kl = key[lo], kh = key[hi];
          if ((kl > kh) == asc) {
            key[lo] = kh; key[hi] = kl;
            const uint16_t tmp = ix[lo]; ix[lo] = ix[hi]; ix[hi] = tmp;
          }
        }
        __syncwarp();
      }
    if (lane == 0) acc += deliver_sorted(c, r, a, k, nullptr, 0, ix);
    __syncwarp();  // the wave's LDS region is reused by its next receiver
  }
  wave_stat_add(c, ST_GOSSIP_ACCEPTED, acc);
  __shared__ uint32_t s_ins[DLV_BLOCK];
  __shared__ uint32_t s_nins;
  for (uint32_t base = blockIdx.x * DLV_BLOCK; base < c.nl; base += gridDim.x * DLV_BLOCK) {
    __syncthreads();  // this workgroup's deliveries (and the previous chunk's inserts) are done
    if (tid == 0) s_nins = 0;
    __syncthreads();
    const uint32_t i = base + tid;
    if (i < c.nl && c.mem[i].ins_rank != 0) s_ins[atomicAdd(&s_nins, 1u)] = c.lo + i;
    __syncthreads();
    const uint32_t nv = s_nins;
    for (uint32_t q = 0; q < nv; ++q) apply_ins_chain(c, s_ins[q]);
  }
  __syncthreads();
  deliver_collect(P, T);
}

// ------------------------------------------------------------------------------- list inserts
// pingMembers.add(nextInt(size), member) (FailureDetectorImpl.java:334-345), in event order: one
// workgroup per viewer with inserts walks the viewer's op chain; each insert shifts the tail right
// by one, tail chunk first.
// The deferred pingMembers.add(nextInt(size), s) ops of viewer v, in event order, by the whole
// workgroup (tail-first parallel shift); every thread of the block must call it.
__device__ void apply_ins_chain(const Ctx& c, uint32_t v) {
  __shared__ uint32_t s_idx, s_s, s_next, s_k;
  MemberDev& m = mem(c, v);
  if (threadIdx.x == 0) s_k = m.ins_rank;
  __syncthreads();
  const uint32_t k = s_k;
  uint32_t* pl = ping_list(c, v);
  uint32_t cur = m.ins_head;
  for (uint32_t q = 0; q < k; ++q) {
    const uint32_t size = m.ping_len;
    if (threadIdx.x == 0) {
      const InsOp op = c.ins[cur];
      s_idx = size > 0 ? next_int(draw(c, v, SWIM_STREAM_PING_INSERT, op.phase, op.minor), size) : 0;
      s_s = op.s;
      s_next = op.next;
    }
    __syncthreads();
    const uint32_t idx = s_idx;
    for (int64_t hi = (int64_t)size; hi > (int64_t)idx; hi -= blockDim.x) {
      int64_t lo = hi - (int64_t)blockDim.x < (int64_t)idx ? (int64_t)idx : hi - (int64_t)blockDim.x;
      int64_t p = lo + threadIdx.x;
      uint32_t val = 0;
      if (p < hi) val = pl[p];
      __syncthreads();
      if (p < hi) pl[p + 1] = val;
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      pl[idx] = s_s;
      m.ping_len = size + 1;
    }
    cur = s_next;
    __syncthreads();
  }
  if (threadIdx.x == 0) m.ins_rank = 0;
  __syncthreads();
}


// ------------------------------------------------------------------------------- phase D
// selectSyncAddress (MembershipProtocolImpl.java:461-472): uniform over seeds U otherMembers by
// seeded rejection sampling.
__device__ inline uint32_t select_sync_address(const Ctx& c, uint32_t v) {
  const MemberDev& m = mem(c, v);
  const uint32_t* a = aux_row(c, v);
  uint32_t count = m.members_size - 1;
  for (uint32_t i = 0; i < c.n_seeds; ++i) {
    uint32_t s = c.seeds[i];
    if (s != v && !(a[s] & A_IN_MEMBERS)) count++;
  }
  if (count == 0) return NONE;
  for (uint32_t i = 0; i < SWIM_SYNC_SELECT_ATTEMPTS; ++i) {
    uint32_t x = next_int(draw(c, v, SWIM_STREAM_SYNC_SELECT, 0, i), c.n);
    if (x != v && ((a[x] & A_IN_MEMBERS) || c.is_seed[x])) return x;
  }
  uint32_t k = next_int(draw(c, v, SWIM_STREAM_SYNC_SELECT, 1, 0), count);
  for (uint32_t x = 0; x < c.n; ++x)
    if (x != v && ((a[x] & A_IN_MEMBERS) || c.is_seed[x])) {
      if (k == 0) return x;
      --k;
    }
  return NONE;
}

// SyncReq.flags: bits 0..2 below; bits 8..31 the number of records the message carries (the
// sender's table size when the message is prepared: the count syncMembership iterates, :491-509)
enum : uint32_t { RQ_INITIAL = 1, RQ_OUTFAIL = 2, RQ_DELIVERED = 4, RQ_RECS_SHIFT = 8 };

// a delivered SYNC / SYNC_ACK joins its receiver's inbox (the receiver is owned by this shard)
__device__ inline void enqueue_sync(const Ctx& c, SyncReq q, SyncReq* items, uint32_t* total, uint32_t* cnt,
                                    uint32_t* recv, uint32_t* recv_cnt, uint32_t cap) {
  q.slot = atomicAdd(&cnt[q.to - c.lo], 1u);
  if (q.slot == 0) recv[atomicAdd(recv_cnt, 1u)] = q.to;
  const uint32_t i = atomicAdd(total, 1u);
  if (i >= cap) { set_err(c, ERR_REQS); return; }
  items[i] = q;
}

__device__ inline void add_req(const Ctx& c, const Bufs& b, uint32_t v, uint32_t to, uint32_t ordinal, bool initial) {
  MemberDev& m = mem(c, v);
  SyncReq q;
  q.from = v; q.to = to; q.ordinal = ordinal; q.slot = 0;
  q.flags = (initial ? RQ_INITIAL : 0) | (m.table_size << RQ_RECS_SHIFT);
  q.content = NONE; q.snap = NONE; q.pad = 0;
  if (initial) m.init_total++;
  if (out_fail(c, v, to, v, SWIM_STREAM_SYNC_OUT, ordinal, 0)) {
    if (initial) m.init_done++;
    return;
  }
  if (!in_pass(c, to, v)) return;  // inbound-blocked at the receiver: silently dropped
  q.flags |= RQ_DELIVERED;
  if (!owned(c, to)) {  // content (this row) travels with the request: k_pack_rows
    const uint32_t d = owner(c, to);
    const uint32_t i = atomicAdd(&b.x->req[d], 1u);
    if (i >= b.tx_req_cap) { set_err(c, ERR_REQS); return; }
    b.tx_reqs[(size_t)d * b.tx_req_cap + i] = q;
    return;
  }
  enqueue_sync(c, q, b.reqs, &b.k->req_total, b.req_cnt, b.req_recv, &b.k->req_recv_cnt, b.req_cap);
}

// doSync (:339-357), FD-triggered SYNCs (:427-442) and start0's initial SYNC to every seed (:250-291)
__device__ inline unsigned long long sync_collect_member(const Ctx& c, const Bufs& b, uint32_t v) {
  const uint32_t i = v - c.lo, t32 = (uint32_t)c.T;
  const bool due = c.sync_next[i] == t32;  // the periodic doSync timer fires (sync_on, phase sync_start)
  const uint32_t fl = c.mflag[i];
  if (!due && !(fl & (MF_FDSYNC | MF_JOIN))) return 0;
  if (due) c.sync_next[i] = t32 + c.S;
  if (fl & MF_FDSYNC) c.mflag[i] = fl & ~MF_FDSYNC;
  MemberDev& m = mem(c, v);
  if (!c.up[v]) { m.fd_sync_cnt = 0; return 0; }
  uint32_t k = 0;
  unsigned long long nsync = 0;
  if (due) {
    uint32_t t = select_sync_address(c, v);
    if (t != NONE) { add_req(c, b, v, t, k++, false); nsync++; }
  }
  for (uint32_t i = 0; i < m.fd_sync_cnt; ++i) {
    add_req(c, b, v, c.fd_sync[(size_t)(v - c.lo) * FD_SYNC_MAX + i], k++, false);
    nsync++;
  }
  m.fd_sync_cnt = 0;
  if (m.join_now) {
    m.init_total = 0;
    m.init_done = 0;
    for (uint32_t i = 0; i < c.n_seeds; ++i) {
      uint32_t s = c.seeds[i];
      if (s != v) { add_req(c, b, v, s, k++, true); nsync++; }
    }
  }
  return nsync;
}


#include "swim_sync.h"


// ------------------------------------------------------------------------------- end of tick
// start0's doFinally (:285-289) for members that joined this tick; graceful leaves complete.
__global__ void k_end_tick(KP, uint32_t n_rx_stops) {
  const Ctx c = pctx(P, T);
  Counters* k = P->b.k;
  Xc* x = P->c.world > 1 ? P->b.x : nullptr;
  const uint32_t* rx_stops = P->b.rx_stops;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // collector blocks freed this tick become allocatable (one workgroup: the counters are read,
  // then rewritten, by the same threads)
  if (blockIdx.x == 0) {
    for (int t = 0; t < NTIER; ++t) {
      const int32_t a0 = c.spill_ctl[t].avail;
      const uint32_t a = a0 > 0 ? (uint32_t)a0 : 0u, f = min(c.spill_ctl[t].freed, c.spill_cap[t] - a);
      for (uint32_t j = threadIdx.x; j < f; j += blockDim.x) c.spill_avail[t][a + j] = c.spill_freed[t][j];
      __syncthreads();
      if (threadIdx.x == 0) {
        c.spill_ctl[t].avail = (int32_t)(a + f);
        c.spill_ctl[t].freed = 0;
      }
    }
  }
  // receipt-bitmap slots requested this tick change owner (no other kernel runs now): zeroed bits,
  // valid from the next tick; the other parity's queue (next tick's) is emptied
  {
    const uint32_t par = (uint32_t)(T & 1);
    const uint32_t nclaim = min(c.gclaim_cnt[par], GSLOTS);
    for (uint32_t q = blockIdx.x; q < nclaim; q += gridDim.x) {
      const uint32_t sl = c.gclaim[par * GSLOTS + q];
      uint32_t* bits = c.gbits + (size_t)sl * c.gwords;
      for (uint32_t w = threadIdx.x; w < c.gwords; w += blockDim.x) bits[w] = 0;
      if (threadIdx.x == 0) {
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
  if (i < n_rx_stops) c.up[rx_stops[i]] = 0;  // graceful leaves completed on other shards
  if (i >= c.nl) return;
  const uint32_t fl = c.mflag[i];
  if (!(fl & (MF_JOIN | MF_LEAVE))) return;
  c.mflag[i] = fl & ~(MF_JOIN | MF_LEAVE);
  const uint32_t v = c.lo + i;
  MemberDev& m = c.mem[i];
  if (m.join_now) {
    m.sync_on = 1;
    m.sync_start = (int64_t)c.T + (m.init_done == m.init_total ? 0 : (int64_t)c.sync_to_ticks);
    m.join_now = 0;
    c.sync_next[i] = next_due(m.sync_start, c.T, c.S);
  }
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
