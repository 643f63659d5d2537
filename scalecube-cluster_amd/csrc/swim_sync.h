// swim_sync.h — phase D kernels: SYNC / SYNC_ACK delivery and the row merge (included inside
// namespace swimdev by swim_phases.h).
//
// syncMembership (MembershipProtocolImpl.java:491-509) runs updateMembership on every record of a
// full table; with a 30 s sync interval N/300 members start a SYNC every tick, so the dominant cost
// of a protocol period is streaming (content row, receiver row) pairs.  It is split in three:
//
//   k_sync_prep      one workgroup: group delivered messages by receiver, canonical inbox order,
//                    snapshot claims for rows that are both read and merged into in this sub-phase
//   k_sync_classify  the HBM stream: one 256-thread workgroup per (message, 4,096-subject chunk),
//                    16 consecutive subjects per thread with 16-B loads; a record is "complex" unless
//                    updateMembership would provably do nothing; complex subjects of a chunk are
//                    block-scan compacted into a pool in subject order
//   k_sync_apply     one workgroup per receiver: lane 0 runs the exact sequential updateMembership on
//                    the complex subjects in (message, chunk, subject) order, then the ALIVE
//                    admissions whose metadata fetch succeeded; a later message to a receiver whose
//                    row already changed this sub-phase is re-classified in-workgroup.

constexpr int SYNC_CHUNK = 4096;
constexpr int CLS_BLOCK = 256;
constexpr int CLS_CPT = SYNC_CHUNK / CLS_BLOCK;  // 16 subjects per thread
constexpr int APPLY_BLOCK = 256;
constexpr int APPLY_CPT = 8;
constexpr int APPLY_TILE = APPLY_BLOCK * APPLY_CPT;

// true unless updateMembership(r1 = content cell) on row cell r0 provably changes nothing
__device__ inline bool sync_complex(uint64_t r1, uint64_t r0, bool self) {
  const uint32_t s1 = c_status(r1);
  const int32_t i1 = c_inc(r1);
  const bool p0 = c_has(r0, B_IN_TABLE);
  const uint32_t s0 = c_status(r0);
  const int32_t i0 = c_inc(r0);
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
__global__ void k_recv_sync(Ctx c, Bufs b, int d2, uint32_t nrx) {
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
__global__ void k_pack_rows(Ctx c, const SyncReq* tx, uint32_t tx_cap, PackPlan plan, uint64_t* out) {
  for (uint32_t d = 0; d < c.world; ++d) {
    for (uint32_t k = blockIdx.x; k < plan.cnt[d]; k += gridDim.x) {
      const SyncReq q = tx[(size_t)d * tx_cap + k];
      const uint64_t* src = row(c, q.from);
      uint64_t* dst = out + (size_t)(plan.off[d] + k) * c.n;
      if (c.n & 1) {  // rows are only 8-B aligned
        for (uint32_t x = threadIdx.x; x < c.n; x += blockDim.x) dst[x] = src[x];
      } else {
        const ulonglong2* s2 = reinterpret_cast<const ulonglong2*>(src);
        ulonglong2* d2 = reinterpret_cast<ulonglong2*>(dst);
        for (uint32_t x = threadIdx.x; x < c.n / 2; x += blockDim.x) d2[x] = s2[x];
      }
    }
  }
}

__device__ __forceinline__ const uint64_t* sync_content(const Ctx& c, const Bufs& b, const SyncReq& q) {
  if (q.content != NONE) return b.rx_rows + (size_t)q.content * c.n;
  const uint32_t si = b.snap_idx[q.from - c.lo];
  return si < b.snap_cap ? b.snap + (size_t)si * c.n : row(c, q.from);
}

__global__ void __launch_bounds__(1024) k_sync_prep(Ctx c, Bufs b, int d2) {
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
}

__global__ void __launch_bounds__(CLS_BLOCK) k_sync_classify(Ctx c, Bufs b, int d2) {
  __shared__ uint32_t s_bits[SYNC_CHUNK / 32];
  const SubPhase p = sub_phase(b, d2);
  const uint32_t ni = *p.nitems;
  const uint32_t chunks = b.chunks, n = c.n;
  unsigned long long recs = 0, msgs = 0, cplx = 0;
  for (uint32_t w = blockIdx.x; w < ni * chunks; w += gridDim.x) {
    const uint32_t i = w / chunks, ch = w - i * chunks;
    const SyncReq q = p.out[i];
    const uint32_t r = q.to, src = q.from;
    const bool remote = q.content != NONE;
    const uint64_t* __restrict__ content = remote ? b.rx_rows + (size_t)q.content * n : row(c, src);
    const uint64_t* __restrict__ rv = row(c, r);
    const uint32_t si = remote ? NONE : b.snap_idx[src - c.lo];
    uint64_t* snapdst = si < b.snap_cap ? b.snap + (size_t)si * n : nullptr;
    if (ch == 0) msgs++;
    // coalesced: load j of lane t covers subjects base + j*512 + 2t, +1 (1 KiB per wave-instruction)
    const uint32_t base = ch * SYNC_CHUNK;
    uint32_t flags = 0;  // bit 2j+h = subject base + j*512 + 2*tid + h
    if (base + SYNC_CHUNK <= n && ((reinterpret_cast<uintptr_t>(content + base) | reinterpret_cast<uintptr_t>(rv + base)) & 15) == 0) {
      ulonglong2 a[CLS_CPT / 2], o[CLS_CPT / 2];
#pragma unroll
      for (int j = 0; j < CLS_CPT / 2; ++j)
        a[j] = *reinterpret_cast<const ulonglong2*>(content + base + j * 2 * CLS_BLOCK + 2 * threadIdx.x);
#pragma unroll
      for (int j = 0; j < CLS_CPT / 2; ++j)
        o[j] = *reinterpret_cast<const ulonglong2*>(rv + base + j * 2 * CLS_BLOCK + 2 * threadIdx.x);
      if (snapdst) {
#pragma unroll
        for (int j = 0; j < CLS_CPT / 2; ++j)
          *reinterpret_cast<ulonglong2*>(snapdst + base + j * 2 * CLS_BLOCK + 2 * threadIdx.x) = a[j];
      }
#pragma unroll
      for (int j = 0; j < CLS_CPT / 2; ++j) {
        const uint32_t x = base + j * 2 * CLS_BLOCK + 2 * threadIdx.x;
        const bool r0 = c_has(a[j].x, B_IN_TABLE), r1 = c_has(a[j].y, B_IN_TABLE);
        recs += (uint32_t)r0 + (uint32_t)r1;
        if (r0 && sync_complex(a[j].x, o[j].x, x == r)) flags |= 1u << (2 * j);
        if (r1 && sync_complex(a[j].y, o[j].y, x + 1 == r)) flags |= 1u << (2 * j + 1);
      }
    } else {
      for (int j = 0; j < CLS_CPT / 2; ++j)
        for (int h = 0; h < 2; ++h) {
          const uint32_t x = base + j * 2 * CLS_BLOCK + 2 * threadIdx.x + h;
          if (x >= n) continue;
          const uint64_t a = content[x];
          if (snapdst) snapdst[x] = a;
          if (c_has(a, B_IN_TABLE)) {
            recs++;
            if (sync_complex(a, rv[x], x == r)) flags |= 1u << (2 * j + h);
          }
        }
    }
    // almost every chunk has no record that can change the receiver: one barrier decides it
    if (!__syncthreads_or(flags != 0)) {
      if (threadIdx.x == 0) b.item_chunk[(size_t)i * chunks + ch] = make_uint2(0, 0);
      continue;
    }
    // rare path: subject-ordered compaction through an LDS bitmap (bit x - base)
    for (uint32_t wdx = threadIdx.x; wdx < SYNC_CHUNK / 32; wdx += CLS_BLOCK) s_bits[wdx] = 0;
    __syncthreads();
    for (int k = 0; k < CLS_CPT; ++k)
      if (flags & (1u << k)) {
        const uint32_t off = (k >> 1) * 2 * CLS_BLOCK + 2 * threadIdx.x + (k & 1);
        atomicOr(&s_bits[off >> 5], 1u << (off & 31));
      }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t total = 0;
      for (uint32_t wdx = 0; wdx < SYNC_CHUNK / 32; ++wdx) total += __popc(s_bits[wdx]);
      uint32_t pb = atomicAdd(&b.k->pool_cursor, total);
      if (pb + total > b.pool_cap) {
        set_err(c, ERR_PEND);
        total = 0;
      } else {
        uint32_t o2 = pb;
        for (uint32_t wdx = 0; wdx < SYNC_CHUNK / 32; ++wdx) {
          uint32_t bits = s_bits[wdx];
          while (bits) {
            const uint32_t bit = __ffs(bits) - 1;
            bits &= bits - 1;
            b.pool[o2++] = base + wdx * 32 + bit;
          }
        }
      }
      b.item_chunk[(size_t)i * chunks + ch] = make_uint2(pb, total);
      atomicAdd(&b.item_total[i], total);
      cplx += total;
    }
    __syncthreads();
  }
  for (int d = 32; d > 0; d >>= 1) recs += __shfl_down(recs, d, 64);
  if ((threadIdx.x & 63) == 0) stat_add(c, ST_SYNC_RECORDS, recs);
  if (threadIdx.x == 0) {
    stat_add(c, ST_MERGE_MSGS, msgs);
    stat_add(c, ST_MERGE_RECORDS, cplx);
  }
}

// In-workgroup merge of one message (used when the receiver's row changed earlier in this
// sub-phase, so the precomputed classification may be stale).  Returns through *s_mod whether any
// record could change the row.
__device__ void merge_row_wg(const Ctx& c, uint32_t v, const uint64_t* __restrict__ content, int reason,
                             uint32_t phase, uint64_t* pend, uint32_t& npend, uint32_t* s_list, uint32_t* s_wave,
                             uint32_t* s_mod) {
  uint64_t* __restrict__ rv = row(c, v);
  const uint32_t n = c.n;
  for (uint32_t base = 0; base < n; base += APPLY_TILE) {
    const uint32_t x0 = base + threadIdx.x * APPLY_CPT;
    uint32_t flags = 0;
    for (int k = 0; k < APPLY_CPT; ++k) {
      const uint32_t x = x0 + k;
      if (x >= n) break;
      const uint64_t a = content[x];
      if (c_has(a, B_IN_TABLE) && sync_complex(a, rv[x], x == v)) flags |= 1u << k;
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
        const uint64_t a = content[x];
        if (update_membership(c, v, x, c_status(a), c_inc(a), reason, phase))
          pend[npend++] = ((uint64_t)x << 32) | (uint32_t)c_inc(a);
      }
    }
    __syncthreads();
  }
}

// SYNC_ACK from `from` (the SYNC receiver) back to `to` (the SYNC sender)
__device__ inline void add_ack(const Ctx& c, const Bufs& b, uint32_t to, uint32_t from, uint32_t rank, bool initial) {
  SyncReq a;
  a.from = from; a.to = to; a.ordinal = rank; a.slot = 0; a.flags = RQ_DELIVERED | (initial ? RQ_INITIAL : 0);
  a.content = NONE; a.pad[0] = a.pad[1] = 0;
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
__global__ void __launch_bounds__(APPLY_BLOCK) k_sync_apply(Ctx c, Bufs b, int d2) {
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
      const uint64_t* content = sync_content(c, b, rq);
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
              const uint64_t a = content[x];
              if (update_membership(c, s, x, c_status(a), c_inc(a), reason, phase))
                pend[npend++] = ((uint64_t)x << 32) | (uint32_t)c_inc(a);
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
