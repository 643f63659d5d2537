// swim_sync.h — phase D kernels: SYNC / SYNC_ACK delivery and the row merge (included inside
// namespace swimdev by swim_phases.h).
//
// syncMembership (MembershipProtocolImpl.java:491-509) runs updateMembership on every record of a
// full table; with a 30 s sync interval N/300 members start a SYNC every tick, so the dominant cost
// of a protocol period is streaming (content row, receiver row) pairs.  It is split in three:
//
//   k_sync_prep      one workgroup: group delivered messages by receiver, canonical inbox order,
//                    snapshot claims for rows that are both read and merged into in this sub-phase
//   k_sync_classify  the HBM stream: one wave per (message, 1,024-subject chunk), 16 subjects per
//                    lane as four 16-B loads of record words per row (content row + receiver row =
//                    8 B per subject), software-pipelined across units; a record is "complex" unless
//                    updateMembership would provably do nothing; complex subjects of a chunk are
//                    block-scan compacted into a pool in subject order
//   k_sync_apply     one workgroup per receiver: lane 0 runs the exact sequential updateMembership on
//                    the complex subjects in (message, chunk, subject) order, then the ALIVE
//                    admissions whose metadata fetch succeeded; a later message to a receiver whose
//                    row already changed this sub-phase is re-classified in-workgroup.

constexpr int SYNC_CHUNK = 1024;                 // subjects per classify unit (one wave)
constexpr int CLS_BLOCK = 256;
constexpr int CLS_LOADS = SYNC_CHUNK / 256;      // 16-B record loads per lane per row
constexpr int APPLY_BLOCK = 256;
constexpr int APPLY_CPT = 8;
constexpr int APPLY_TILE = APPLY_BLOCK * APPLY_CPT;

// true unless updateMembership(r1 = content record) on the row record r0 provably changes nothing
__device__ inline bool sync_complex(uint32_t r1, uint32_t r0, bool self) {
  const uint32_t s1 = r_status(r1);
  const int32_t i1 = r_inc(r1);
  const bool p0 = r_in_table(r0);
  const uint32_t s0 = r_status(r0);
  const int32_t i0 = r_inc(r0);
  const bool r0_leaving = p0 && s0 == SWIM_LEAVING;
  if (!r0_leaving && !is_overrides(s1, i1, p0, s0, i0)) return false;  // :593-602
  // an identical LEAVING record over a LEAVING row is a no-op put, except on the viewer's own row,
  // where it re-runs onSelfMemberDetected (:604-607)
  if (r0_leaving && s1 == SWIM_LEAVING && i1 == i0 && !self) return false;
  return true;
}

__device__ inline void sort_reqs(SyncReq* a, uint32_t n) {
  for (uint32_t i = 1; i < n; ++i) {
    SyncReq x = a[i];
    int32_t j = (int32_t)i - 1;
    while (j >= 0 && (a[j].from > x.from || (a[j].from == x.from && a[j].ordinal > x.ordinal))) { a[j + 1] = a[j]; --j; }
    a[j + 1] = x;
  }
}

struct SubPhase {  // the SYNC (d2 = 0) or SYNC_ACK (d2 = 1) buffers
  SyncReq* items;
  uint32_t total;
  uint32_t* recv;
  uint32_t nrecv;
  uint32_t* cnt;
  uint32_t* start;
  SyncReq* out;
  uint32_t* nitems;
};

__device__ inline SubPhase sub_phase(const Bufs& b, int d2) {
  SubPhase p;
  if (!d2) {
    p.items = b.reqs; p.total = min(b.k->req_total, b.req_cap); p.recv = b.req_recv; p.nrecv = b.k->req_recv_cnt;
    p.cnt = b.req_cnt; p.start = b.req_start; p.out = b.reqs_out; p.nitems = &b.k->req_cursor;
  } else {
    p.items = b.acks; p.total = min(b.k->ack_total, b.req_cap); p.recv = b.ack_recv; p.nrecv = b.k->ack_recv_cnt;
    p.cnt = b.ack_cnt; p.start = b.ack_start; p.out = b.acks_out; p.nitems = &b.k->ack_cursor;
  }
  return p;
}

// SYNCs / SYNC_ACKs arriving from other shards (content row = rx_rows[k]) join their inboxes
__global__ void k_recv_sync(KP, int d2, uint32_t nrx) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nrx; k += gridDim.x * blockDim.x) {
    SyncReq q = b.rx_reqs[k];
    q.content = k;
    if (!d2) enqueue_sync(c, q, b.reqs, &b.k->req_total, b.req_cnt, b.req_recv, &b.k->req_recv_cnt, b.req_cap);
    else enqueue_sync(c, q, b.acks, &b.k->ack_total, b.ack_cnt, b.ack_recv, &b.k->ack_recv_cnt, b.req_cap);
  }
}

// content rows of this shard's outgoing SYNC / SYNC_ACKs, packed per destination in tx order (the
// sender's table when the message is prepared, prepareSyncDataMsg :485-489)
struct PackPlan {
  uint32_t cnt[MAXW];
  uint32_t off[MAXW];  // first packed row of destination d
};
__global__ void k_pack_rows(Ctx c, const SyncReq* tx, uint32_t tx_cap, PackPlan plan, uint32_t* out) {
  for (uint32_t d = 0; d < c.world; ++d) {
    for (uint32_t k = blockIdx.x; k < plan.cnt[d]; k += gridDim.x) {
      const SyncReq q = tx[(size_t)d * tx_cap + k];
      const uint32_t* src = rec_row(c, q.from);
      uint32_t* dst = out + (size_t)(plan.off[d] + k) * c.n;
      if (c.n & 3) {  // rows are only 4-B aligned
        for (uint32_t x = threadIdx.x; x < c.n; x += blockDim.x) dst[x] = src[x];
      } else {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (uint32_t x = threadIdx.x; x < c.n / 4; x += blockDim.x) d4[x] = s4[x];
      }
    }
  }
}

// the record row a SYNC / SYNC_ACK carries: received copy, snapshot, or the sender's live row
__device__ __forceinline__ const uint32_t* sync_content(const Ctx& c, const Bufs& b, const SyncReq& q) {
  if (q.content != NONE) return b.rx_rows + (size_t)q.content * c.n;
  const uint32_t si = b.snap_idx[q.from - c.lo];
  return si < b.snap_cap ? b.snap + (size_t)si * c.n : rec_row(c, q.from);
}

__global__ void __launch_bounds__(1024) k_sync_prep(KP, int d2) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  __shared__ uint32_t s_cursor;
  const SubPhase p = sub_phase(b, d2);
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  // release the previous sub-phase's snapshot claims
  const uint32_t prev = min(*b.snap_cnt, b.snap_cap);
  for (uint32_t i = tid; i < prev; i += nt) b.snap_idx[b.snap_list[i] - c.lo] = NONE;
  if (tid == 0) s_cursor = 0;
  __syncthreads();
  if (tid == 0) *b.snap_cnt = 0;
  // one contiguous inbox per receiver
  for (uint32_t i = tid; i < p.nrecv; i += nt) {
    const uint32_t r = p.recv[i] - c.lo;
    p.start[r] = atomicAdd(&s_cursor, p.cnt[r]);
  }
  __syncthreads();
  if (tid == 0) *p.nitems = s_cursor;
  for (uint32_t i = tid; i < p.total; i += nt) {
    const SyncReq q = p.items[i];
    p.out[p.start[q.to - c.lo] + q.slot] = q;
  }
  __syncthreads();
  // canonical order inside an inbox: (sender, ordinal)
  for (uint32_t i = tid; i < p.nrecv; i += nt) {
    const uint32_t r = p.recv[i] - c.lo;
    sort_reqs(p.out + p.start[r], p.cnt[r]);
  }
  __syncthreads();
  // message content = the sender's table when the message was prepared: a sender that is itself
  // merged into during this sub-phase gets its row snapshotted by k_sync_classify
  const uint32_t ni = s_cursor;
  for (uint32_t i = tid; i < ni; i += nt) {
    b.item_total[i] = 0;
    if (p.out[i].content != NONE) continue;  // content arrived from another shard: already a copy
    const uint32_t src = p.out[i].from, sl = src - c.lo;
    if (p.cnt[sl] == 0) continue;
    if (atomicCAS(&b.snap_idx[sl], NONE, NONE - 1) == NONE) {
      const uint32_t slot = atomicAdd(b.snap_cnt, 1u);
      if (slot >= b.snap_cap) { set_err(c, ERR_SNAP); b.snap_idx[sl] = NONE; continue; }
      b.snap_list[slot] = src;
      b.snap_idx[sl] = slot;
    }
  }
  __syncthreads();
  __threadfence_block();
  // every message records its sender's snapshot slot (classify reads it with the header)
  for (uint32_t i = tid; i < ni; i += nt) {
    SyncReq& q = p.out[i];
    q.snap = q.content != NONE ? NONE : b.snap_idx[q.from - c.lo];
  }
}

// One (message, chunk) unit per wave: 64 lanes x 16 subjects = SYNC_CHUNK subjects, i.e. four
// 16-B loads of record words per lane from the content row and four from the receiver row.  Each
// wave owns a contiguous range of units, so consecutive units share the message header (loaded once
// per message), and walks it with a one-deep software pipeline: the next unit's rows are in flight
// while the current one is classified.  Complex subjects are compacted into the pool in subject
// order with a ballot and a wave scan (no workgroup barriers).
struct ClsHdr {
  const uint32_t* content;
  const uint32_t* rv;
  uint32_t* snapdst;
  uint32_t i, r;
};

__device__ __forceinline__ void cls_hdr(const Ctx& c, const Bufs& b, const SubPhase& p, uint32_t i, ClsHdr& h) {
  const SyncReq q = p.out[i];
  const bool remote = q.content != NONE;
  h.content = remote ? b.rx_rows + (size_t)q.content * c.n : rec_row(c, q.from);
  h.rv = rec_row(c, q.to);
  h.snapdst = q.snap < b.snap_cap ? b.snap + (size_t)q.snap * c.n : nullptr;
  h.i = i;
  h.r = q.to;
}

__device__ __forceinline__ void cls_rows(const Ctx& c, const ClsHdr& h, uint32_t ch, uint32_t lane, uint4* a, uint4* o) {
  const uint32_t n = c.n, base = ch * SYNC_CHUNK;
  const bool full = base + SYNC_CHUNK <= n && ((reinterpret_cast<uintptr_t>(h.content + base) |
                                                reinterpret_cast<uintptr_t>(h.rv + base)) & 15) == 0;
  if (full) {
#pragma unroll
    for (int j = 0; j < CLS_LOADS; ++j) a[j] = *reinterpret_cast<const uint4*>(h.content + base + j * 256 + 4 * lane);
#pragma unroll
    for (int j = 0; j < CLS_LOADS; ++j) o[j] = *reinterpret_cast<const uint4*>(h.rv + base + j * 256 + 4 * lane);
    return;
  }
  // ragged tail of a row (N not a multiple of SYNC_CHUNK) or rows only 4-B aligned
#pragma unroll
  for (int j = 0; j < CLS_LOADS; ++j) {
    uint32_t av[4], ov[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t x = base + j * 256 + 4 * lane + q;
      av[q] = x < n ? h.content[x] : 0u;  // 0 = not in the table: never complex
      ov[q] = x < n ? h.rv[x] : 0u;
    }
    a[j] = make_uint4(av[0], av[1], av[2], av[3]);
    o[j] = make_uint4(ov[0], ov[1], ov[2], ov[3]);
  }
}

// prof (profiled launches only): {messages merged, complex records} of this launch
__global__ void __launch_bounds__(CLS_BLOCK) k_sync_classify(KP, int d2, unsigned long long* prof) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  const SubPhase p = sub_phase(b, d2);
  const uint32_t ni = *p.nitems;
  const uint32_t chunks = b.chunks, n = c.n;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * (CLS_BLOCK / 64) + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * (CLS_BLOCK / 64);
  const uint64_t total = (uint64_t)ni * chunks;
  const uint32_t u0 = (uint32_t)(total * wid / nw), u1 = (uint32_t)(total * (wid + 1) / nw);
  unsigned long long recs = 0, cplx = 0;
  __shared__ unsigned long long s_recs[CLS_BLOCK / 64];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    stat_add(c, ST_MERGE_MSGS, ni);
    if (prof) prof[0] = ni;
  }
  if (u0 < u1) {
    ClsHdr hc, hn;
    uint4 a[CLS_LOADS], o[CLS_LOADS], an[CLS_LOADS], on[CLS_LOADS];
    cls_hdr(c, b, p, u0 / chunks, hc);
    cls_rows(c, hc, u0 - hc.i * chunks, lane, a, o);
    hn = hc;
    for (uint32_t u = u0; u < u1; ++u) {
      const uint32_t ch = u - hc.i * chunks;
      const bool more = u + 1 < u1;
      if (more) {
        const uint32_t i2 = (u + 1) / chunks;
        if (i2 != hn.i) cls_hdr(c, b, p, i2, hn);
        cls_rows(c, hn, u + 1 - i2 * chunks, lane, an, on);
      }
      const uint32_t base = ch * SYNC_CHUNK;
      if (hc.snapdst) {
#pragma unroll
        for (int j = 0; j < CLS_LOADS; ++j) {
          const uint32_t av[4] = {a[j].x, a[j].y, a[j].z, a[j].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t x = base + j * 256 + 4 * lane + q;
            if (x < n) hc.snapdst[x] = av[q];
          }
        }
      }
      uint32_t flags = 0;  // bit 4j+q = subject base + j*256 + 4*lane + q
      uint32_t diff = 0;
#pragma unroll
      for (int j = 0; j < CLS_LOADS; ++j) {
        diff |= (a[j].x ^ o[j].x) | (a[j].y ^ o[j].y) | (a[j].z ^ o[j].z) | (a[j].w ^ o[j].w);
        recs += (a[j].x >> 31) + (a[j].y >> 31) + (a[j].z >> 31) + (a[j].w >> 31);
      }
      // identical records never change the row (isOverrides(equal) is false and an identical
      // LEAVING over LEAVING is a no-op) except on the viewer's own subject: the fast path of a
      // converged cluster, where nearly every lane of nearly every unit compares equal
      const uint32_t off = hc.r - base;
      const bool self_here = off < SYNC_CHUNK && ((off & 255u) >> 2) == lane;
      if (diff != 0 || self_here) {
#pragma unroll
        for (int j = 0; j < CLS_LOADS; ++j) {
          const uint32_t x = base + j * 256 + 4 * lane;
          const uint32_t av[4] = {a[j].x, a[j].y, a[j].z, a[j].w};
          const uint32_t ov[4] = {o[j].x, o[j].y, o[j].z, o[j].w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (r_in_table(av[q]) && sync_complex(av[q], ov[q], x + q == hc.r)) flags |= 1u << (4 * j + q);
        }
      }
      uint2 res = make_uint2(0, 0);
      if (__ballot(flags != 0)) {
        // rare path: subject order = (j, lane, q); one wave scan of the four per-j counts
        uint64_t cnt = 0;
#pragma unroll
        for (int j = 0; j < CLS_LOADS; ++j) cnt |= (uint64_t)__popc((flags >> (4 * j)) & 0xfu) << (16 * j);
        uint64_t incl = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint64_t y = __shfl_up(incl, d, 64);
          if (lane >= (uint32_t)d) incl += y;
        }
        const uint64_t tot = __shfl(incl, 63, 64);
        const uint64_t excl = incl - cnt;
        uint32_t t = 0, jbase[CLS_LOADS];
#pragma unroll
        for (int j = 0; j < CLS_LOADS; ++j) { jbase[j] = t; t += (uint32_t)(tot >> (16 * j)) & 0xffffu; }
        uint32_t pb = 0;
        if (lane == 0) pb = atomicAdd(&b.k->pool_cursor, t);
        pb = __shfl(pb, 0, 64);
        if (pb + t > b.pool_cap) {
          if (lane == 0) set_err(c, ERR_PEND);
          t = 0;
        } else {
#pragma unroll
          for (int j = 0; j < CLS_LOADS; ++j) {
            uint32_t o2 = pb + jbase[j] + ((uint32_t)(excl >> (16 * j)) & 0xffffu);
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (flags & (1u << (4 * j + q))) b.pool[o2++] = base + j * 256 + 4 * lane + q;
          }
        }
        res = make_uint2(pb, t);
        if (lane == 0 && t) atomicAdd(&b.item_total[hc.i], t);
        cplx += t;
      }
      if (lane == 0) b.item_chunk[(size_t)hc.i * chunks + ch] = res;
      if (more) {
        hc = hn;
#pragma unroll
        for (int j = 0; j < CLS_LOADS; ++j) { a[j] = an[j]; o[j] = on[j]; }
      }
    }
  }
  // one counter update per workgroup (4,096 waves on one replicated counter would serialise)
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) recs += __shfl_down(recs, d, 64);
  if (lane == 0) s_recs[threadIdx.x >> 6] = recs;
  if (lane == 0 && cplx) {
    stat_add(c, ST_MERGE_RECORDS, cplx);
    if (prof) atomicAdd(prof + 1, cplx);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < CLS_BLOCK / 64; ++w) t += s_recs[w];
    stat_add(c, ST_SYNC_RECORDS, t);
  }
}

// In-workgroup merge of one message (used when the receiver's row changed earlier in this
// sub-phase, so the precomputed classification may be stale).  Returns through *s_mod whether any
// record could change the row.
__device__ void merge_row_wg(const Ctx& c, uint32_t v, const uint32_t* __restrict__ content, int reason,
                             uint32_t phase, uint64_t* pend, uint32_t& npend, uint32_t* s_list, uint32_t* s_wave,
                             uint32_t* s_mod) {
  const uint32_t* __restrict__ rv = rec_row(c, v);
  const uint32_t n = c.n;
  for (uint32_t base = 0; base < n; base += APPLY_TILE) {
    const uint32_t x0 = base + threadIdx.x * APPLY_CPT;
    uint32_t flags = 0;
    for (int k = 0; k < APPLY_CPT; ++k) {
      const uint32_t x = x0 + k;
      if (x >= n) break;
      const uint32_t a = content[x];
      if (r_in_table(a) && sync_complex(a, rv[x], x == v)) flags |= 1u << k;
    }
    uint32_t total;
    const uint32_t off = block_exclusive_scan<APPLY_BLOCK>((uint32_t)__popc(flags), s_wave, &total);
    if (total == 0) continue;
    uint32_t o = off;
    for (int k = 0; k < APPLY_CPT; ++k)
      if (flags & (1u << k)) s_list[o++] = x0 + k;
    __syncthreads();
    if (threadIdx.x == 0) {
      *s_mod = 1;
      for (uint32_t i = 0; i < total; ++i) {
        const uint32_t x = s_list[i];
        const uint32_t a = content[x];
        if (update_membership(c, v, x, r_status(a), r_inc(a), reason, phase))
          pend[npend++] = ((uint64_t)x << 32) | (uint32_t)r_inc(a);
      }
    }
    __syncthreads();
  }
}

// SYNC_ACK from `from` (the SYNC receiver) back to `to` (the SYNC sender)
__device__ inline void add_ack(const Ctx& c, const Bufs& b, uint32_t to, uint32_t from, uint32_t rank, bool initial) {
  SyncReq a;
  a.from = from; a.to = to; a.ordinal = rank; a.slot = 0; a.flags = RQ_DELIVERED | (initial ? RQ_INITIAL : 0);
  a.content = NONE; a.snap = NONE; a.pad = 0;
  if (!owned(c, to)) {  // content (this row after the SYNC merges) travels with the ack
    const uint32_t d = owner(c, to);
    const uint32_t i = atomicAdd(&b.x->ack[d], 1u);
    if (i >= b.tx_req_cap) { set_err(c, ERR_REQS); return; }
    b.tx_acks[(size_t)d * b.tx_req_cap + i] = a;
    return;
  }
  enqueue_sync(c, a, b.acks, &b.k->ack_total, b.ack_cnt, b.ack_recv, &b.k->ack_recv_cnt, b.req_cap);
}

// D1 (d2 = 0): onSync at each receiver, then its SYNC_ACKs.  D2 (d2 = 1): the SYNC_ACK merge at
// the original senders (MembershipProtocolImpl.java:363-415).
__global__ void __launch_bounds__(APPLY_BLOCK) k_sync_apply(KP, int d2) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  __shared__ uint32_t s_list[APPLY_TILE];
  __shared__ uint32_t s_wave[APPLY_BLOCK / 64 + 1];
  __shared__ uint32_t s_mod;
  const SubPhase p = sub_phase(b, d2);
  const uint32_t phase = d2 ? SWIM_PHASE_SYNCACK : SWIM_PHASE_SYNC;
  const uint32_t chunks = b.chunks;
  uint64_t* pend = b.pend + (size_t)blockIdx.x * c.n;
  for (uint32_t i = blockIdx.x; i < p.nrecv; i += gridDim.x) {
    const uint32_t s = p.recv[i];
    const uint32_t k = p.cnt[s - c.lo];
    const uint32_t first = p.start[s - c.lo];
    if (threadIdx.x == 0) {
      mem(c, s).ev_minor = 0;
      mem(c, s).fetch_ctr = 0;
      s_mod = 0;
    }
    __syncthreads();
    for (uint32_t q = 0; q < k; ++q) {
      const SyncReq rq = p.out[first + q];
      const uint32_t* content = sync_content(c, b, rq);
      const int reason = (d2 && (rq.flags & RQ_INITIAL)) ? R_INITIAL_SYNC : R_SYNC;
      uint32_t npend = 0;
      const uint32_t mod = s_mod;
      __syncthreads();  // every lane has read s_mod before lane 0 may set it
      if (mod == 0) {  // precomputed classification is exact: the row is unchanged
        if (threadIdx.x == 0 && b.item_total[first + q] != 0) {
          const uint2* ic = b.item_chunk + (size_t)(first + q) * chunks;
          for (uint32_t ch = 0; ch < chunks; ++ch) {
            const uint2 e = ic[ch];
            if (e.y) s_mod = 1;
            for (uint32_t j = 0; j < e.y; ++j) {
              const uint32_t x = b.pool[e.x + j];
              const uint32_t a = content[x];
              if (update_membership(c, s, x, r_status(a), r_inc(a), reason, phase))
                pend[npend++] = ((uint64_t)x << 32) | (uint32_t)r_inc(a);
            }
          }
        }
      } else {
        merge_row_wg(c, s, content, reason, phase, pend, npend, s_list, s_wave, &s_mod);
      }
      if (threadIdx.x == 0) {
        for (uint32_t j = 0; j < npend; ++j)
          apply_alive(c, s, (uint32_t)(pend[j] >> 32), (int32_t)(uint32_t)pend[j], reason, phase);
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (!d2) {
        for (uint32_t q = 0; q < k; ++q) {
          const SyncReq rq = p.out[first + q];
          if (out_fail(c, s, rq.from, s, SWIM_STREAM_SYNCACK_OUT, q, 0)) continue;
          if (!in_pass(c, rq.from, s)) continue;
          add_ack(c, b, rq.from, s, q, (rq.flags & RQ_INITIAL) != 0);
        }
      } else {
        // start0's initial-sync completion counts the acks of its INITIAL SYNCs (:270-284)
        uint32_t init = 0;
        for (uint32_t q = 0; q < k; ++q) init += (p.out[first + q].flags & RQ_INITIAL) ? 1u : 0u;
        mem(c, s).init_done += init;
        stat_add(c, ST_SYNC_ACKS, k);
      }
      p.cnt[s - c.lo] = 0;
    }
    __syncthreads();
  }
}
