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
//                    8 B per subject), units whose two rows both equal the reference row there (the
//                    exact block witness, Ctx.bdiff) skipped without a row load; a record is
//                    "complex" unless updateMembership would provably do nothing; complex subjects of
//                    a chunk are wave-scan compacted into a pool in subject order
//   k_sync_apply     one workgroup per receiver: lane 0 runs the exact sequential updateMembership on
//                    the complex subjects in (message, chunk, subject) order, then the ALIVE
//                    admissions whose metadata fetch succeeded; a later message to a receiver whose
//                    row already changed this sub-phase is re-classified in-workgroup.

#ifndef CLS_MINWAVES
#define CLS_MINWAVES 4  // waves per SIMD the classify kernels are register-limited to
#endif
#ifndef CLS_SKIPZERO
#define CLS_SKIPZERO 0  // timing experiment only: skip the stores of empty chunk results (NOT exact)
#endif
#ifndef CLS_REV
#define CLS_REV 1       // SYNC classify also classifies the reverse (SYNC_ACK) direction
#endif
#ifndef CLS_WITNESS
#define CLS_WITNESS 1   // 1: units the block witness proves identical are skipped (0: stream all;
                        // 2, 3: timing experiments only, NOT exact)
#endif
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
  uint2* desc;
  SyncReq* out;
  uint32_t* nitems;
};

__device__ inline SubPhase sub_phase(const Bufs& b, int d2) {
  SubPhase p;
  if (!d2) {
    p.items = b.reqs; p.total = min(b.k->req_total, b.req_cap); p.recv = b.req_recv; p.nrecv = b.k->req_recv_cnt;
    p.cnt = b.req_cnt; p.start = b.req_start; p.desc = b.req_desc; p.out = b.reqs_out; p.nitems = &b.k->req_cursor;
  } else {
    p.items = b.acks; p.total = min(b.k->ack_total, b.req_cap); p.recv = b.ack_recv; p.nrecv = b.k->ack_recv_cnt;
    p.cnt = b.ack_cnt; p.start = b.ack_start; p.desc = b.ack_desc; p.out = b.acks_out; p.nitems = &b.k->ack_cursor;
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
// Packed rows are copied in 16-KiB chunks, one workgroup per (row, chunk): a handful of 256-KiB
// rows per exchange would otherwise leave most CUs idle (one workgroup per row ran at ~2 GB/s).
constexpr uint32_t PACK_CHUNK = 4096;  // record words per unit
__global__ void __launch_bounds__(256) k_pack_rows(Ctx c, const SyncReq* tx, uint32_t tx_cap, PackPlan plan,
                                                   uint32_t tot, uint32_t* out) {
  const uint32_t per_row = (c.n + PACK_CHUNK - 1) / PACK_CHUNK;
  for (uint32_t u = blockIdx.x; u < tot * per_row; u += gridDim.x) {
    const uint32_t row = u / per_row, ch = u - row * per_row;
    uint32_t d = 0;  // destination of packed row `row` (plan.off is the running sum of plan.cnt)
    while (d + 1 < c.world && row >= plan.off[d] + plan.cnt[d]) ++d;
    const SyncReq q = tx[(size_t)d * tx_cap + (row - plan.off[d])];
    const uint32_t x0 = ch * PACK_CHUNK, len = min(PACK_CHUNK, c.n - x0);
    const uint32_t* src = rec_row(c, q.from) + x0;
    uint32_t* dst = out + (size_t)row * c.n + x0;
    if (c.n & 3) {  // rows are only 4-B aligned
      for (uint32_t x = threadIdx.x; x < len; x += blockDim.x) dst[x] = src[x];
    } else {
      const uint4* s4 = reinterpret_cast<const uint4*>(src);
      uint4* d4 = reinterpret_cast<uint4*>(dst);
      for (uint32_t x = threadIdx.x; x < len / 4; x += blockDim.x) d4[x] = s4[x];
    }
  }
}

// the record row a SYNC / SYNC_ACK carries: received copy, snapshot, or the sender's live row
__device__ __forceinline__ const uint32_t* sync_content(const Ctx& c, const Bufs& b, const SyncReq& q) {
  if (q.content != NONE) return b.rx_rows + (size_t)q.content * c.n;
  const uint32_t si = b.snap_idx[q.from - c.lo];
  return si < b.snap_cap ? b.snap + (size_t)si * c.n : rec_row(c, q.from);
}

// k_sync_prep: the sub-phase's delivered messages -> one contiguous inbox per receiver in canonical
// (sender, ordinal) order, snapshot claims for senders that are merged into in the same sub-phase.
// Messages are staged in LDS (receivers found through an LDS hash, inbox order sorted as LDS index
// permutations), so the single workgroup makes ~3 dependent rounds of global accesses instead of
// one per step; sub-phases larger than the LDS stage take the global path.
constexpr uint32_t PREP_CAP = 2048;    // messages (and receivers) staged in LDS
constexpr uint32_t PREP_HASH = 4096;   // receiver hash slots (power of two, >= 2 x PREP_CAP)
constexpr int PREP_BLOCK = 1024;

__device__ __forceinline__ uint32_t prep_slot(uint32_t id) { return (id * 2654435761u) >> 20; }  // 12 bits

__device__ __forceinline__ uint32_t prep_find(const uint32_t* hkey, const uint32_t* hval, uint32_t id) {
  for (uint32_t h = prep_slot(id);; h = (h + 1) & (PREP_HASH - 1)) {
    const uint32_t k = hkey[h];
    if (k == id) return hval[h];
    if (k == NONE) return NONE;
  }
}

__device__ void sync_prep_global(const Ctx& c, const Bufs& b, const SubPhase& p, int d2) {
  __shared__ uint32_t s_cursor;
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) s_cursor = 0;
  __syncthreads();
  // one contiguous inbox per receiver
  for (uint32_t i = tid; i < p.nrecv; i += nt) {
    const uint32_t r = p.recv[i] - c.lo;
    p.start[r] = atomicAdd(&s_cursor, p.cnt[r]);
    p.desc[i] = make_uint2(p.start[r], p.cnt[r]);
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
  // merged into during this sub-phase gets its row snapshotted
  const uint32_t ni = s_cursor;
  for (uint32_t i = tid; i < ni; i += nt) {
    b.item_total[i] = 0;
    if (!d2) b.rev_total[i] = 0;
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

__device__ void sync_prep_lds(const Ctx& c, const Bufs& b, const SubPhase& p, int d2) {
  __shared__ SyncReq s_q[PREP_CAP];          // staged messages (64 KiB)
  __shared__ uint32_t s_perm[PREP_CAP];      // inbox position -> staged message
  __shared__ uint32_t s_rid[PREP_CAP];       // receiver index -> member
  __shared__ uint32_t s_start[PREP_CAP + 1]; // receiver index -> message count, then inbox start
  __shared__ uint32_t s_snap[PREP_CAP];      // receiver index -> snapshot slot of its row
  __shared__ uint32_t s_hkey[PREP_HASH], s_hval[PREP_HASH];
  __shared__ uint32_t s_wave[PREP_BLOCK / 64 + 1];
  __shared__ uint32_t s_nsnap;
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  const uint32_t ni = p.total, nr = p.nrecv;
  // release the previous sub-phase's snapshot claims; their loads overlap the staging loads
  // (the claims below are made after several barriers; *snap_cnt is rewritten at the end)
  const uint32_t prev = min(*b.snap_cnt, b.snap_cap);
  for (uint32_t h = tid; h < PREP_HASH; h += nt) s_hkey[h] = NONE;
  if (tid == 0) s_nsnap = 0;
  __syncthreads();
  const uint32_t rel = tid < prev ? b.snap_list[tid] : NONE;
  for (uint32_t i = tid; i < ni; i += nt) s_q[i] = p.items[i];
  for (uint32_t i = tid; i < nr; i += nt) {
    const uint32_t id = p.recv[i];
    s_rid[i] = id;
    s_start[i] = p.cnt[id - c.lo];
    s_snap[i] = NONE;
    for (uint32_t h = prep_slot(id);; h = (h + 1) & (PREP_HASH - 1))
      if (atomicCAS(&s_hkey[h], NONE, id) == NONE) { s_hval[h] = i; break; }
  }
  if (rel != NONE) b.snap_idx[rel - c.lo] = NONE;
  for (uint32_t i = tid + nt; i < prev; i += nt) b.snap_idx[b.snap_list[i] - c.lo] = NONE;  // snap_cap > block
  if (tid >= nr && tid < 2 * PREP_BLOCK) s_start[tid] = 0;  // scan padding
  if (tid + PREP_BLOCK >= nr && tid + PREP_BLOCK < PREP_CAP) s_start[tid + PREP_BLOCK] = 0;
  __syncthreads();
  // inbox starts: exclusive scan of the counts, two receivers per thread
  const uint32_t c0 = s_start[2 * tid], c1 = s_start[2 * tid + 1];
  uint32_t total;
  const uint32_t ex = block_exclusive_scan<PREP_BLOCK>(c0 + c1, s_wave, &total);
  s_start[2 * tid] = ex;
  s_start[2 * tid + 1] = ex + c0;
  if (tid == 0) { s_start[nr] = total; *p.nitems = total; }
  __syncthreads();
  for (uint32_t i = tid; i < nr; i += nt) {
    p.start[s_rid[i] - c.lo] = s_start[i];
    p.desc[i] = make_uint2(s_start[i], s_start[i + 1] - s_start[i]);
  }
  for (uint32_t i = tid; i < ni; i += nt) {
    const uint32_t ri = prep_find(s_hkey, s_hval, s_q[i].to);
    s_perm[s_start[ri] + s_q[i].slot] = i;
  }
  __syncthreads();
  // canonical order inside an inbox: (sender, ordinal)
  for (uint32_t ri = tid; ri < nr; ri += nt) {
    uint32_t* a = s_perm + s_start[ri];
    const uint32_t k = s_start[ri + 1] - s_start[ri];
    for (uint32_t x = 1; x < k; ++x) {
      const uint32_t v = a[x];
      const uint32_t vf = s_q[v].from, vo = s_q[v].ordinal;
      int32_t y = (int32_t)x - 1;
      while (y >= 0 && (s_q[a[y]].from > vf || (s_q[a[y]].from == vf && s_q[a[y]].ordinal > vo))) {
        a[y + 1] = a[y];
        --y;
      }
      a[y + 1] = v;
    }
  }
  __syncthreads();
  // snapshot claims: message content = the sender's table when the message was prepared; a sender
  // that is itself merged into during this sub-phase gets its row snapshotted
  for (uint32_t pos = tid; pos < total; pos += nt) {
    const SyncReq& q = s_q[s_perm[pos]];
    if (q.content != NONE) continue;  // content arrived from another shard: already a copy
    const uint32_t rs = prep_find(s_hkey, s_hval, q.from);
    if (rs == NONE || atomicCAS(&s_snap[rs], NONE, NONE - 1) != NONE) continue;
    const uint32_t slot = atomicAdd(&s_nsnap, 1u);
    if (slot >= b.snap_cap) { set_err(c, ERR_SNAP); s_snap[rs] = NONE; continue; }
    s_snap[rs] = slot;
    b.snap_list[slot] = q.from;
    b.snap_idx[q.from - c.lo] = slot;
  }
  __syncthreads();
  for (uint32_t pos = tid; pos < total; pos += nt) {
    SyncReq q = s_q[s_perm[pos]];
    uint32_t sn = NONE;
    if (q.content == NONE) {
      const uint32_t rs = prep_find(s_hkey, s_hval, q.from);
      if (rs != NONE && s_snap[rs] < b.snap_cap) sn = s_snap[rs];
    }
    q.snap = sn;
    p.out[pos] = q;
    b.item_total[pos] = 0;
    if (!d2) b.rev_total[pos] = 0;
  }
  if (tid == 0) *b.snap_cnt = min(s_nsnap, b.snap_cap);
}

// copy_snaps (SYNC_ACK sub-phase of an unsharded engine, where no classify launch streams the ack
// rows): copy the claimed rows here, before any SYNC_ACK merge can change them
__global__ void __launch_bounds__(PREP_BLOCK) k_sync_prep(KP, int d2, int copy_snaps) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  const SubPhase p = sub_phase(b, d2);
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  if (p.total <= PREP_CAP && p.nrecv <= PREP_CAP) {
    sync_prep_lds(c, b, p, d2);  // releases the previous sub-phase's snapshot claims itself
  } else {
    // release the previous sub-phase's snapshot claims
    const uint32_t prev = min(*b.snap_cnt, b.snap_cap);
    for (uint32_t i = tid; i < prev; i += nt) b.snap_idx[b.snap_list[i] - c.lo] = NONE;
    __syncthreads();
    if (tid == 0) *b.snap_cnt = 0;
    __syncthreads();
    sync_prep_global(c, b, p, d2);
  }
  if (!copy_snaps) return;
  __syncthreads();
  __threadfence_block();
  const uint32_t ns = min(*b.snap_cnt, b.snap_cap), n = c.n;
  for (uint32_t k = 0; k < ns; ++k) {
    const uint32_t* src = rec_row(c, b.snap_list[k]);
    uint32_t* dst = b.snap + (size_t)k * n;
    if ((n & 3) == 0) {
      for (uint32_t x = tid; x < n / 4; x += nt)
        reinterpret_cast<uint4*>(dst)[x] = reinterpret_cast<const uint4*>(src)[x];
    } else {
      for (uint32_t x = tid; x < n; x += nt) dst[x] = src[x];
    }
  }
}

// One (message, chunk) unit per wave: 64 lanes x 16 subjects = SYNC_CHUNK subjects, i.e. four
// 16-B loads of record words per lane from the content row and four from the receiver row.  Each
// wave owns a contiguous range of units, so consecutive units share the message header (loaded once
// per message), and walks it with a one-deep software pipeline: the next unit's rows are in flight
// while the current one is classified.  Complex subjects are compacted into the pool in subject
// order with a ballot and a wave scan (no workgroup barriers).
//
// SYNC_ACK reuse.  The SYNC_ACK answering a local SYNC s -> r merges r's row into s's row: the same
// two rows with the roles swapped.  The SYNC launch (d2 = 0) therefore classifies both directions
// from one load of the pair and keeps the reverse result (rev_chunk / rev_total).  The
// SYNC_ACK launch reuses it for an ack whose two rows no SYNC merge of this tick touched (row_mod,
// stamped by k_sync_apply), which is exact: classification is a pure function of the two rows.
struct ClsHdr {
  const uint32_t* content;
  const uint32_t* rv;
  const uint32_t* bdc;  // block witness of the content row (local content only), else nullptr
  const uint32_t* bdv;  // block witness of the receiver row
  uint32_t* snapdst;
  uint32_t i, r, s;
  uint32_t rev;  // d2 = 0: 1 = also classify the reverse direction (a local SYNC)
  uint32_t d1;   // d2 = 1: the SYNC whose reverse classification this ack reuses, or NONE
};

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// the header is wave-uniform: keep it in scalar registers (the row loads need the VGPRs)
// (speculative = true: message i may lie beyond the sub-phase's items, so nothing is read through
// the header's ids; the SYNC_ACK reuse check is left out)
__device__ __forceinline__ void cls_hdr(const Ctx& c, const Bufs& b, const SubPhase& p, int d2, uint32_t i, ClsHdr& h,
                                        bool speculative = false) {
  SyncReq q = p.out[i];
  q.from = uni(q.from); q.to = uni(q.to); q.content = uni(q.content); q.snap = uni(q.snap); q.pad = uni(q.pad);
  const bool remote = q.content != NONE;
  h.content = remote ? b.rx_rows + (size_t)q.content * c.n : rec_row(c, q.from);
  h.rv = rec_row(c, q.to);
  h.bdc = remote ? nullptr : c.bdiff + (size_t)(q.from - c.lo) * c.blocks;
  h.bdv = c.bdiff + (size_t)(q.to - c.lo) * c.blocks;
  h.snapdst = q.snap < b.snap_cap ? b.snap + (size_t)q.snap * c.n : nullptr;
  h.i = i;
  h.r = q.to;
  h.s = q.from;
  h.rev = (CLS_REV && !d2 && !remote) ? 1u : 0u;
  h.d1 = NONE;
  if (d2 && !speculative && q.pad != 0 && !remote) {
    const uint32_t t = (uint32_t)c.T;
    if (uni(b.row_mod[q.from - c.lo]) != t && uni(b.row_mod[q.to - c.lo]) != t) h.d1 = q.pad - 1;
  }
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

// wave-uniform: compact the subjects flagged in `flags` (bit 4j+q = subject base + j*256 + 4*lane + q)
// into the pool in subject order; returns (pool base, count)
__device__ __forceinline__ uint2 cls_compact(const Ctx& c, const Bufs& b, uint32_t flags, uint32_t base,
                                             uint32_t lane) {
  if (!__ballot(flags != 0)) return make_uint2(0, 0);
  // subject order = (j, lane, q); one wave scan of the four per-j counts
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
    return make_uint2(pb, 0);
  }
#pragma unroll
  for (int j = 0; j < CLS_LOADS; ++j) {
    uint32_t o2 = pb + jbase[j] + ((uint32_t)(excl >> (16 * j)) & 0xffffu);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (flags & (1u << (4 * j + q))) b.pool[o2++] = base + j * 256 + 4 * lane + q;
  }
  return make_uint2(pb, t);
}

__device__ __forceinline__ bool lane_holds(uint32_t subject, uint32_t base, uint32_t lane) {
  const uint32_t off = subject - base;
  return off < SYNC_CHUNK && ((off & 255u) >> 2) == lane;
}

// a viewer's own subject x in the unit starting at base is complex even when both records equal ref
// there (an identical LEAVING re-runs onSelfMemberDetected, sync_complex)
__device__ __forceinline__ bool self_complex(const Ctx& c, uint32_t x, uint32_t base) {
  if (x - base >= (uint32_t)SYNC_CHUNK) return false;
  const uint32_t rf = c.ref[x];
  return r_in_table(rf) && r_status(rf) == SWIM_LEAVING;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_down(x, d, 64);
  return x;
}

// D2 = 0: the SYNC launch k_sync_classify (streams every message's two rows, both directions);
// D2 = 1: the SYNC_ACK launch k_ack_classify (reuses the SYNC launch's reverse results, streams only
// acks whose rows changed).  A unit whose two rows both equal ref throughout the block (block
// witness counts 0, Ctx.bdiff) holds identical records and is not streamed: its results are empty
// (the two self subjects excepted, checked on ref).  prof (profiled launches only): {units streamed,
// complex records, units in the launch}.
template <int D2>
__device__ __forceinline__ void classify_body(const Params* __restrict__ P, uint64_t T, unsigned long long* prof) {
  constexpr int d2 = D2;
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  const SubPhase p = sub_phase(b, d2);
  const uint32_t chunks = b.chunks, n = c.n;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * (CLS_BLOCK / 64) + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * (CLS_BLOCK / 64);
  // units are dealt grid-stride (wave w: units w, w + nw, ...); the first header is loaded
  // speculatively, in parallel with the item count
  const uint32_t i0 = wid / chunks;
  ClsHdr hc;
  if (i0 < b.req_cap) cls_hdr(c, b, p, d2, i0, hc, true);
  const uint32_t ni = *p.nitems;
  const uint32_t total = ni * chunks;
  uint32_t cplx = 0, streamed = 0, skipped = 0;
  if (wid < total) {
    if (d2) cls_hdr(c, b, p, d2, i0, hc);  // now a valid item: add the SYNC_ACK reuse check
    for (uint32_t u = wid; u < total; u += nw) {
      const uint32_t i = u / chunks;
      if (i != hc.i) cls_hdr(c, b, p, d2, i, hc);
      const uint32_t ch = u - i * chunks;
      const uint32_t base = ch * SYNC_CHUNK;
      if (CLS_WITNESS && hc.d1 == NONE && !hc.snapdst && hc.bdc) {
        const uint32_t dc = CLS_WITNESS == 3 ? 0u : uni(hc.bdc[ch]), dv = CLS_WITNESS == 3 ? 0u : uni(hc.bdv[ch]);
        if ((dc | dv) == 0 && !self_complex(c, hc.r, base) && !(hc.rev && self_complex(c, hc.s, base))) {
          if (lane == 0 && CLS_WITNESS != 2) {
            b.item_chunk[(size_t)hc.i * chunks + ch] = make_uint2(0, 0);
            if (hc.rev) b.rev_chunk[(size_t)hc.i * chunks + ch] = make_uint2(0, 0);
          }
          ++skipped;
          continue;
        }
      }
      uint4 a[CLS_LOADS], o[CLS_LOADS];
      if (hc.d1 == NONE || hc.snapdst) cls_rows(c, hc, ch, lane, a, o);
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
      if (hc.d1 != NONE) {
        // SYNC_ACK whose classification the SYNC launch already made
        if (lane == 0) {
          b.item_chunk[(size_t)hc.i * chunks + ch] = b.rev_chunk[(size_t)hc.d1 * chunks + ch];
          if (ch == 0) {
            const uint32_t t = b.rev_total[hc.d1];
            b.item_total[hc.i] = t;
            cplx += t;
          }
        }
        continue;
      }
      ++streamed;
      uint32_t flags = 0, rflags = 0;
      uint32_t diff = 0;
#pragma unroll
      for (int j = 0; j < CLS_LOADS; ++j)
        diff |= (a[j].x ^ o[j].x) | (a[j].y ^ o[j].y) | (a[j].z ^ o[j].z) | (a[j].w ^ o[j].w);
      // identical records never change the row (isOverrides(equal) is false and an identical
      // LEAVING over LEAVING is a no-op) except on the viewer's own subject
      const bool self_here = lane_holds(hc.r, base, lane);
      const bool rself_here = hc.rev && lane_holds(hc.s, base, lane);
      if (diff != 0 || self_here || rself_here) {
#pragma unroll
        for (int j = 0; j < CLS_LOADS; ++j) {
          const uint32_t x = base + j * 256 + 4 * lane;
          const uint32_t av[4] = {a[j].x, a[j].y, a[j].z, a[j].w};
          const uint32_t ov[4] = {o[j].x, o[j].y, o[j].z, o[j].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (r_in_table(av[q]) && sync_complex(av[q], ov[q], x + q == hc.r)) flags |= 1u << (4 * j + q);
            if (hc.rev && r_in_table(ov[q]) && sync_complex(ov[q], av[q], x + q == hc.s))
              rflags |= 1u << (4 * j + q);
          }
        }
      }
      const uint2 res = cls_compact(c, b, flags, base, lane);
      if (lane == 0 && (!CLS_SKIPZERO || res.y)) {
        b.item_chunk[(size_t)hc.i * chunks + ch] = res;
        if (res.y) atomicAdd(&b.item_total[hc.i], res.y);
      }
      cplx += res.y;
      if (hc.rev) {
        const uint2 rres = cls_compact(c, b, rflags, base, lane);
        if (lane == 0 && (!CLS_SKIPZERO || rres.y)) {
          b.rev_chunk[(size_t)hc.i * chunks + ch] = rres;
          if (rres.y) atomicAdd(&b.rev_total[hc.i], rres.y);
        }
      }
    }
  }
  // the message record counts (sync_records) are taken from the headers by k_sync_apply; only
  // non-zero counts are added (thousands of waves skip every unit: one atomic each on the same
  // address would serialise the launch), the unit total is stored once
  (void)skipped;
  if (lane == 0 && (cplx || streamed)) {
    if (cplx) stat_add(c, ST_MERGE_RECORDS, cplx);
    if (streamed) stat_add(c, ST_MERGE_MSGS, streamed);
    if (prof) {
      if (streamed) atomicAdd(prof, (unsigned long long)streamed);
      if (cplx) atomicAdd(prof + 1, (unsigned long long)cplx);
    }
  }
  if (prof && wid == 0 && lane == 0) prof[2] = total;
}

__global__ void __launch_bounds__(CLS_BLOCK, CLS_MINWAVES) k_sync_classify(KP, unsigned long long* prof) {
  classify_body<0>(P, T, prof);
}
__global__ void __launch_bounds__(CLS_BLOCK, CLS_MINWAVES) k_ack_classify(KP) { classify_body<1>(P, T, nullptr); }

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
// `d1` = 1 + index of the SYNC being answered when its classify also classified this ack (0 = none)
__device__ inline void add_ack(const Ctx& c, const Bufs& b, uint32_t to, uint32_t from, uint32_t rank, bool initial,
                               uint32_t d1) {
  SyncReq a;
  a.from = from; a.to = to; a.ordinal = rank; a.slot = 0;
  a.flags = RQ_DELIVERED | (initial ? RQ_INITIAL : 0) | (mem(c, from).table_size << RQ_RECS_SHIFT);
  a.content = NONE; a.snap = NONE; a.pad = d1;
  if (!owned(c, to)) {  // content (this row after the SYNC merges) travels with the ack
    a.pad = 0;
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
// classified = 0 (SYNC_ACK sub-phase of an unsharded engine: no k_ack_classify launch): an ack takes
// the SYNC launch's reverse classification when its two rows are unchanged since (row_mod), and is
// classified in-workgroup (merge_row_wg) otherwise.
__global__ void __launch_bounds__(APPLY_BLOCK) k_sync_apply(KP, int d2, int classified) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  __shared__ uint32_t s_list[APPLY_TILE];
  __shared__ uint32_t s_wave[APPLY_BLOCK / 64 + 1];
  __shared__ uint32_t s_mod;
  __shared__ unsigned long long s_recs;
  __shared__ uint32_t s_iP[APPLY_BLOCK], s_iS[APPLY_BLOCK], s_iR[APPLY_BLOCK];
  const SubPhase p = sub_phase(b, d2);
  const uint32_t phase = d2 ? SWIM_PHASE_SYNCACK : SWIM_PHASE_SYNC;
  const uint32_t chunks = b.chunks;
  uint64_t* pend = b.pend + (size_t)blockIdx.x * c.n;
  for (uint32_t i = blockIdx.x; i < p.nrecv; i += gridDim.x) {
    const uint32_t s = p.recv[i];
    const uint2 dsc = p.desc[i];  // loaded with the receiver id: no dependent cnt / start lookup
    const uint32_t first = dsc.x, k = dsc.y;
    if (threadIdx.x == 0) {
      mem(c, s).ev_minor = 0;
      mem(c, s).fetch_ctr = 0;
      s_mod = 0;
      s_recs = 0;
    }
    __syncthreads();
    for (uint32_t q = 0; q < k; ++q) {
      const SyncReq rq = p.out[first + q];
      const uint32_t tot_q = b.item_total[first + q];  // issued with the header (stable since classify)
      const uint32_t* content = sync_content(c, b, rq);
      const int reason = (d2 && (rq.flags & RQ_INITIAL)) ? R_INITIAL_SYNC : R_SYNC;
      uint32_t npend = 0;
      const uint32_t mod = s_mod;
      const bool own = d2 && !classified;  // this kernel classifies the ack
      uint32_t d1 = NONE;
      if (own && rq.pad != 0 && rq.content == NONE && b.row_mod[rq.from - c.lo] != (uint32_t)c.T &&
          b.row_mod[s - c.lo] != (uint32_t)c.T)
        d1 = rq.pad - 1;
      __syncthreads();  // every lane has read s_mod before lane 0 may set it
      if (mod == 0 && (!own || d1 != NONE)) {  // precomputed classification is exact: the row is unchanged
        const uint32_t it = d1 != NONE ? d1 : first + q;
        const uint32_t tot = d1 != NONE ? b.rev_total[it] : tot_q;
        if (threadIdx.x == 0 && tot != 0) {
          const uint2* ic = (d1 != NONE ? b.rev_chunk : b.item_chunk) + (size_t)it * chunks;
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
        s_recs += rq.flags >> RQ_RECS_SHIFT;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (!d2) {
        for (uint32_t q = 0; q < k; ++q) {
          const SyncReq rq = p.out[first + q];
          if (out_fail(c, s, rq.from, s, SWIM_STREAM_SYNCACK_OUT, q, 0)) continue;
          if (!in_pass(c, rq.from, s)) continue;
          add_ack(c, b, rq.from, s, q, (rq.flags & RQ_INITIAL) != 0, CLS_REV && rq.content == NONE ? first + q + 1 : 0);
        }
        if (s_mod) b.row_mod[s - c.lo] = (uint32_t)c.T;  // invalidates the reverse classifications
      } else {
        // start0's initial-sync completion counts the acks of its INITIAL SYNCs (:270-284)
        uint32_t init = 0;
        for (uint32_t q = 0; q < k; ++q) init += (p.out[first + q].flags & RQ_INITIAL) ? 1u : 0u;
        mem(c, s).init_done += init;
        stat_add(c, ST_SYNC_ACKS, k);
      }
      p.cnt[s - c.lo] = 0;
      stat_add(c, ST_SYNC_RECORDS, s_recs);
    }
    __syncthreads();
    // this sub-phase's pingMembers inserts of s (its ADDED events, all made by this workgroup)
    apply_ins_batch<APPLY_BLOCK, true>(c, s, threadIdx.x, s_iP, s_iS, s_iR);
  }
}
