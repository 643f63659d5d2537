// swim_sync.h — phase D kernels: SYNC / SYNC_ACK delivery and the row merge (included inside
// namespace swimdev by swim_phases.h).
//
// syncMembership (MembershipProtocolImpl.java:491-509) runs updateMembership on every record of a
// full table; with a 30 s sync interval N/300 members start a SYNC every tick, so the dominant cost
// of a protocol period is comparing (content row, receiver row) pairs.  Messages enter paged
// per-receiver inboxes as they are collected (enqueue_sync), so a sub-phase needs no grouping pass:
//
//   k_sync_classify  the row stream: one wave per (message, 1,024-subject chunk), 16 subjects per
//                    lane as four 16-B loads of record words per row (content row + receiver row =
//                    8 B per subject), units whose two rows both equal the reference row there (the
//                    exact block witness, Ctx.bdiff) skipped without a row load; a record is
//                    "complex" unless updateMembership would provably do nothing; complex subjects of
//                    a chunk are wave-scan compacted into a pool in subject order.  The SYNC launch
//                    also classifies the SYNC_ACK direction of every local message, and copies the
//                    content rows that need a snapshot (claimed during collection, sflag_set).
//   k_sync_apply     one workgroup per receiver: its inbox in canonical (sender, ordinal) order (an
//                    in-LDS rank sort of its few messages), then lane 0 runs the exact sequential
//                    updateMembership on the complex subjects in (message, chunk, subject) order,
//                    then the ALIVE admissions whose metadata fetch succeeded; a later message to a
//                    receiver whose row already changed this sub-phase is re-classified in-workgroup.
//                    The SYNC launch sends the SYNC_ACKs and snapshots the acker rows that the
//                    SYNC_ACK sub-phase both reads and merges into.

#ifndef CLS_MINWAVES
#define CLS_MINWAVES 4  // waves per SIMD the classify kernels are register-limited to
#endif
#ifndef CLS_REV
#define CLS_REV 1       // SYNC classify also classifies the reverse (SYNC_ACK) direction
#endif
#ifndef CLS_WITNESS
#define CLS_WITNESS 1   // 1: units the block witness proves identical are skipped (0: stream all)
#endif
static_assert(CLS_WITNESS == 0 || CLS_WITNESS == 1, "CLS_WITNESS is an exact 0 / 1 switch");
static_assert(CLS_REV == 0 || CLS_REV == 1, "CLS_REV is an exact 0 / 1 switch");
constexpr int SYNC_CHUNK = 1024;                 // subjects per classify unit (one wave)
constexpr int CLS_BLOCK = 256;
constexpr int CLS_LOADS = SYNC_CHUNK / 256;      // 16-B record loads per lane per row
constexpr int APPLY_BLOCK = 256;
constexpr int APPLY_CPT = 8;
constexpr int APPLY_TILE = APPLY_BLOCK * APPLY_CPT;
constexpr uint32_t SY_INBOX = 2048;  // messages one receiver's sub-phase inbox holds (sy_max x 64)

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

// E2 / E3.  The content rows of this shard's outgoing SYNCs (d2 = 0) / SYNC_ACKs (d2 = 1) — the
// sender's table when the message is prepared (prepareSyncDataMsg :485-489) — are packed per
// destination in tx order into tx_rows[d2]; each header learns its row (SyncReq.content), which is
// how the receiver finds it.  Offsets come from this shard's own counters: no host round trip.
// Rows are copied in 4-KiB chunks, one workgroup per (row, chunk): a handful of 256-KiB rows per
// exchange would otherwise leave most CUs idle.
constexpr uint32_t PACK_CHUNK = 1024;  // record words per unit (4 KiB: a dozen rows still spread over ~1,000 workgroups)
__global__ void __launch_bounds__(256) k_pack_rows(KP, int d2) {
  // (the counts live in LDS and the few Ctx fields are read directly: a dynamically indexed count
  // array or a Ctx copy would live in scratch)
  const Bufs& b = P->b;
  const uint32_t n = P->c.n, lo = P->c.lo, world = P->c.world, rank = P->c.rank;
  const uint32_t* recs = P->c.recs;
  __shared__ uint32_t s_n[MAXW];
  if (threadIdx.x < (uint32_t)MAXW) {
    const uint32_t d = threadIdx.x;
    const uint32_t* cnt = d2 ? b.x->ack : b.x->req;
    s_n[d] = d < world && d != rank ? min(cnt[d], b.tx_req_cap) : 0u;
  }
  __syncthreads();
  uint32_t total = 0;
  for (uint32_t d = 0; d < (uint32_t)MAXW; ++d) total += s_n[d];
  if (total > b.row_cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(P->c.err, ERR_REQS);
  SyncReq* tx = d2 ? b.tx_acks : b.tx_reqs;
  uint32_t* out = b.tx_rows[d2];
  const uint32_t per_row = (n + PACK_CHUNK - 1) / PACK_CHUNK;
  for (uint32_t u = blockIdx.x; u < total * per_row; u += gridDim.x) {
    const uint32_t row = u / per_row, ch = u - row * per_row;
    uint32_t k = row, d = 0;
    while (k >= s_n[d]) { k -= s_n[d]; ++d; }
    SyncReq* q = tx + (size_t)d * b.tx_req_cap + k;
    const uint32_t fl = q->flags;
    const bool fits = row < b.row_cap;
    // a SYNC_ACK k_ack_delay deferred travels later (content NONE: the receiver skips it)
    if (ch == 0 && threadIdx.x == 0) q->content = fits && !(fl & RQ_DEFER) ? row : NONE;
    if (!fits || (fl & RQ_DEFER)) continue;
    const uint32_t x0 = ch * PACK_CHUNK, len = min(PACK_CHUNK, n - x0);
    // a delayed message's content is its park slot (the row as it was when the message was prepared)
    const uint32_t* src = ((fl & RQ_PARKED) ? b.park + (size_t)q->snap * n : recs + (size_t)(q->from - lo) * n) + x0;
    uint32_t* dst = out + (size_t)row * n + x0;
    if (n & 3) {  // rows are only 4-B aligned
      for (uint32_t x = threadIdx.x; x < len; x += blockDim.x) dst[x] = src[x];
    } else {
      const uint4* s4 = reinterpret_cast<const uint4*>(src);
      uint4* d4 = reinterpret_cast<uint4*>(dst);
      for (uint32_t x = threadIdx.x; x < len / 4; x += blockDim.x) d4[x] = s4[x];
    }
  }
}

// SYNCs / SYNC_ACKs other shards sent to receivers owned here join their inboxes; a message's
// content row is row `content` of the sender's shard p: SyncReq.content = p * row_cap + content
// (wave-uniform trip count: enqueue_sync's page discipline wants every lane of the wave)
__global__ void k_recv_sync(KP, int d2) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  __shared__ uint32_t s_n[MAXW];
  const uint32_t total = peer_counts(c, b, d2 ? XK_ACK : XK_REQ, b.tx_req_cap, s_n);
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t k0 = blockIdx.x * blockDim.x + (threadIdx.x - lane); k0 < total; k0 += gridDim.x * blockDim.x) {
    uint32_t k = k0 + lane;
    SyncReq q{};
    bool valid = k < total;
    if (valid) {
      const uint32_t p = peer_of(s_n, k);
      q = ld_peer(b.peers->hdr[d2][p] + (size_t)c.rank * b.tx_req_cap + k);
      // a marker (pack_inject): a deferred SYNC_ACK for q.to leaves this tick — merged into in the
      // SYNC_ACK sub-phase, no lone-SYNC_ACK shortcut for another ack it gets
      if (!d2 && (q.flags & RQ_PHANTOM)) sflag_set(c, b, q.to - c.lo, SF_SENT | SF_MULTI);
      valid = q.content != NONE;  // its row did not fit the sender's tx_rows (ERR_REQS is set there), or deferred
      q.content = p * b.row_cap + q.content;
      // a delayed SYNC_ACK's receiver is merged into in this SYNC_ACK sub-phase (see k_sync_delay)
      if (valid && d2 && (q.flags & RQ_PARKED)) sflag_set(c, b, q.to - c.lo, SF_SENT);
    }
    enqueue_sync(c, b, d2, q, valid);
  }
}

// RCCL only: the content rows other ranks packed for this one, pulled over xGMI into rx_rows[d2]
// (row p * row_cap + content), one workgroup per (row, chunk)
__global__ void __launch_bounds__(256) k_pull_rows(KP, int d2) {
  const Ctx c = pctx(P, T);
  const Bufs b = P->b;
  const Peers* pr = b.peers;
  __shared__ uint32_t s_n[MAXW];
  const uint32_t total = peer_counts(c, b, d2 ? XK_ACK : XK_REQ, b.tx_req_cap, s_n);
  const uint32_t per_row = (c.n + PACK_CHUNK - 1) / PACK_CHUNK;
  for (uint32_t u = blockIdx.x; u < total * per_row; u += gridDim.x) {
    uint32_t k = u / per_row;
    const uint32_t ch = u - k * per_row;
    const uint32_t p = peer_of(s_n, k);
    const uint32_t row = ld_peer_u32(&pr->hdr[d2][p][(size_t)c.rank * b.tx_req_cap + k].content);
    if (row >= b.row_cap) continue;
    const uint32_t x0 = ch * PACK_CHUNK, len = min(PACK_CHUNK, c.n - x0);
    const uint32_t* src = pr->rows[d2][p] + (size_t)row * c.n + x0;
    uint32_t* dst = pr->rx_rows[d2] + ((size_t)p * b.row_cap + row) * c.n + x0;
    if (c.n & 1) {  // rows are only 4-B aligned
      for (uint32_t x = threadIdx.x; x < len; x += blockDim.x) dst[x] = ld_peer_u32(src + x);
    } else {
      const uint64_t* s8 = reinterpret_cast<const uint64_t*>(src);
      uint64_t* d8 = reinterpret_cast<uint64_t*>(dst);
      for (uint32_t x = threadIdx.x; x < len / 2; x += blockDim.x) d8[x] = ld_peer(s8 + x);
    }
  }
}

// where a received message's content row is: row `content % row_cap` of shard content / row_cap.
// Also evaluated for the speculative header of no message (classify's look-ahead), whose content
// is arbitrary: only arithmetic on such a pointer, which is never read, so no load may fault.
__device__ __forceinline__ const uint32_t* remote_row(const Ctx& c, const Bufs& b, int d2, uint32_t content) {
  if (!b.peers) return c.recs;  // unsharded: nothing arrives from other shards
  const uint32_t p = content / b.row_cap;
  if (p >= (uint32_t)MAXW) return c.recs;
  return b.peers->rows_in[d2][p] + (size_t)(content - p * b.row_cap) * c.n;
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
  uint32_t i, r, s;
  uint32_t rev;  // d2 = 0: 1 = also classify the reverse direction (a local SYNC)
  uint32_t pad;  // d2 = 1: 1 + the SYNC whose reverse classification this ack may reuse, or 0
  uint32_t ph;   // a phantom (deferred SYNC_ACK): nothing to classify
};

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// the header is wave-uniform: keep it in scalar registers (the row loads need the VGPRs)
// (speculative = true: message i may lie beyond the sub-phase's items, so nothing is read through
// the header's ids; the SYNC_ACK reuse check is left out)
__device__ __forceinline__ void cls_hdr(const Ctx& c, const Bufs& b, const SyInbox& p, int d2, uint32_t i, ClsHdr& h) {
  SyncReq q = p.items[i];
  q.from = uni(q.from); q.to = uni(q.to); q.content = uni(q.content); q.pad = uni(q.pad);
  const bool remote = q.content != NONE;
  const bool parked = !remote && (q.flags & RQ_PARKED);  // (uniform: the header is)
  h.ph = !d2 && !remote && (q.flags & RQ_PHANTOM) ? 1u : 0u;
  if (h.ph) q.from = q.to;  // (its sender may live on another shard: no pointer into its row)
  h.content = remote ? remote_row(c, b, d2, q.content) : parked ? park_row(c, b, q.snap) : rec_row(c, q.from);
  h.rv = rec_row(c, q.to);
  h.bdc = remote || parked ? nullptr : c.bdiff + (size_t)(q.from - c.lo) * c.blocks;
  h.bdv = c.bdiff + (size_t)(q.to - c.lo) * c.blocks;
  h.i = i;
  h.r = q.to;
  h.s = q.from;
  h.rev = (CLS_REV && !d2 && !remote && !parked) ? 1u : 0u;
  h.pad = q.pad;
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
  const SyInbox p = sy_inbox(b, d2);
  uint2* const ichunk = d2 ? b.ack_chunk : b.item_chunk;
  uint32_t* const itot = d2 ? b.ack_ctot : b.item_total;
  const uint32_t chunks = b.chunks, n = c.n;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * (CLS_BLOCK / 64) + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * (CLS_BLOCK / 64);
  // units are dealt grid-stride (wave w: units w, w + nw, ...); the first header is loaded
  // speculatively, in parallel with the item count
  const uint32_t i0 = wid / chunks;
  ClsHdr hc;
  if (i0 < b.req_cap) cls_hdr(c, b, p, d2, i0, hc);
  const uint32_t ni = min(*p.total, b.req_cap);
  const uint32_t total = ni * chunks;
  uint32_t cplx = 0, streamed = 0, skipped = 0;
  if (wid < total) {
    for (uint32_t u = wid; u < total; u += nw) {
      const uint32_t i = u / chunks;
      if (i != hc.i) cls_hdr(c, b, p, d2, i, hc);
      const uint32_t ch = u - i * chunks;
      const uint32_t base = ch * SYNC_CHUNK;
      if (hc.ph) {  // a phantom merges nothing (k_sync_apply skips it)
        if (lane == 0) ichunk[(size_t)hc.i * chunks + ch] = make_uint2(0, 0);
        continue;
      }
      // one batch of loads that depend only on the header: the receiver's snapshot slot (a SYNC
      // receiver that also sent a SYNC this tick, sflag_set: this launch copies its row, streamed
      // here before any merge, into the slot; the SYNC_ACK launch needs none), the SYNC_ACK reuse
      // stamps, both block counts and the self subjects' ref words
      const bool local = hc.bdc != nullptr;
      const bool r_here = hc.r - base < (uint32_t)SYNC_CHUNK, s_here = hc.rev && hc.s - base < (uint32_t)SYNC_CHUNK;
      uint32_t rmf = 0, rmt = 0, dc = 1, dv = 1, rfr = 0, rfs = 0;
      if (d2 && local && hc.pad) {
        rmf = b.row_mod[hc.s - c.lo];
        rmt = b.row_mod[hc.r - c.lo];
      }
      if (CLS_WITNESS && local) {
        dc = hc.bdc[ch];
        dv = hc.bdv[ch];
      }
      if (r_here) rfr = c.ref[hc.r];
      if (s_here) rfs = c.ref[hc.s];
      const uint32_t t32 = (uint32_t)c.T;
      const uint32_t d1 = (d2 && local && hc.pad && uni(rmf) != t32 && uni(rmt) != t32) ? hc.pad - 1 : NONE;
      // an identical record on a viewer's own subject is complex when it is LEAVING (sync_complex)
      const auto leaving = [](uint32_t rf) { return r_in_table(rf) && r_status(rf) == SWIM_LEAVING; };
      if (CLS_WITNESS && d1 == NONE && local) {
        if ((uni(dc) | uni(dv)) == 0 && !(r_here && leaving(uni(rfr))) && !(s_here && leaving(uni(rfs)))) {
          if (lane == 0) {
            ichunk[(size_t)hc.i * chunks + ch] = make_uint2(0, 0);
            if (hc.rev) b.rev_chunk[(size_t)hc.i * chunks + ch] = make_uint2(0, 0);
          }
          ++skipped;
          continue;
        }
      }
      uint4 a[CLS_LOADS], o[CLS_LOADS];
      if (d1 == NONE) cls_rows(c, hc, ch, lane, a, o);
      if (d1 != NONE) {
        // SYNC_ACK whose classification the SYNC launch already made
        if (lane == 0) {
          ichunk[(size_t)hc.i * chunks + ch] = b.rev_chunk[(size_t)d1 * chunks + ch];
          if (ch == 0) {
            const uint32_t t = b.rev_total[d1];
            itot[hc.i] = t;
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
      if (lane == 0) {
        ichunk[(size_t)hc.i * chunks + ch] = res;
        if (res.y) atomicAdd(&itot[hc.i], res.y);
      }
      cplx += res.y;
      if (hc.rev) {
        const uint2 rres = cls_compact(c, b, rflags, base, lane);
        if (lane == 0) {
          b.rev_chunk[(size_t)hc.i * chunks + ch] = rres;
          if (rres.y) atomicAdd(&b.rev_total[hc.i], rres.y);
        }
      }
    }
  }
  // the message record counts (sync_records) are taken from the headers by k_sync_apply; the work
  // counters are kept only on profiled launches (same-address atomics from every streaming wave
  // would serialise the launch), the unit total is stored once
  (void)skipped;
  if (prof && lane == 0 && (cplx || streamed)) {
    if (streamed) atomicAdd(prof, (unsigned long long)streamed);
    if (cplx) atomicAdd(prof + 1, (unsigned long long)cplx);
  }
  if (prof && wid == 0 && lane == 0) prof[2] = total;
}

__global__ void __launch_bounds__(CLS_BLOCK, CLS_MINWAVES) k_sync_classify(KP, unsigned long long* prof) {
  classify_body<0>(P, T, prof);
}
__global__ void __launch_bounds__(CLS_BLOCK, CLS_MINWAVES) k_ack_classify(KP) { classify_body<1>(P, T, nullptr); }

// ---- message content under concurrent merges (lazy snapshots).  A SYNC carries its sender's row
// as it was before the SYNC merges (prepareSyncDataMsg :485-489), a SYNC_ACK its acker's row as it
// was before the SYNC_ACK merges.  A member whose row is read as such content by another receiver's
// workgroup while its own workgroup merges into it (it both sent and received this tick: sflag
// SENT | RECV, which claimed a snapshot slot at collection) copies its row into the slot just
// before its FIRST change of the sub-phase and then publishes snap_ready = tick << 2 | phase bit;
// a row that no merge changes is never copied (every quiet tick).  A reader takes the slot once it
// is published, else the live row — and re-checks the flag after the read: a value read while the
// flag was still unpublished predates every change (the writer changes nothing before publishing).
struct Content {
  const uint32_t* live;
  const uint32_t* snap;   // the sender's slot, or nullptr when no merge can change the live row now
  const uint32_t* ready;  // its snap_ready word
  uint32_t want;
};
__device__ __forceinline__ uint32_t snap_want(const Ctx& c, int d2) { return ((uint32_t)c.T << 2) | (d2 ? 2u : 1u); }
// a slot holds the row (n words) and, after it, the row's block-witness counts (blocks words)
__device__ __forceinline__ uint32_t* snap_slot(const Ctx& c, const Bufs& b, uint32_t slot) {
  return b.snap + (size_t)slot * (c.n + c.blocks);
}
__device__ __forceinline__ bool snap_published(const Content& k) {
  return __hip_atomic_load(k.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == k.want;
}
__device__ inline uint32_t content_at(const Content& k, uint32_t x) {
  if (!k.snap) return k.live[x];
  if (snap_published(k)) return k.snap[x];
  const uint32_t v = k.live[x];
  __threadfence();  // the value is in before the flag is read again
  return snap_published(k) ? k.snap[x] : v;
}
// the content of message q (received rows, the sender's slot or its live row)
__device__ __forceinline__ Content msg_content(const Ctx& c, const Bufs& b, const SyncReq& q, int d2) {
  if (q.content != NONE) return Content{remote_row(c, b, d2, q.content), nullptr, nullptr, 0};
  if (q.flags & RQ_PARKED) return Content{park_row(c, b, q.snap), nullptr, nullptr, 0};  // delayed, parked here
  const uint32_t i = q.from - c.lo;
  const uint32_t si = (d2 ? b.ack_snap : b.snap_idx)[i];
  if (si >= b.snap_cap) return Content{rec_row(c, q.from), nullptr, nullptr, 0};
  return Content{rec_row(c, q.from), snap_slot(c, b, si), b.snap_ready + i, snap_want(c, d2)};
}

// the copy of row s (and its witness counts) into its slot before its first change in sub-phase d2,
// then the publication (every thread of the workgroup calls it)
__device__ inline void copy_row(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t n);
__device__ inline void lazy_snapshot(const Ctx& c, const Bufs& b, uint32_t s, uint32_t slot, int d2) {
  uint32_t* dst = snap_slot(c, b, slot);
  copy_row(rec_row(c, s), dst, c.n);
  const uint32_t* bd = c.bdiff + (size_t)(s - c.lo) * c.blocks;
  for (uint32_t k = threadIdx.x; k < c.blocks; k += blockDim.x) dst[c.n + k] = bd[k];
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(b.snap_ready + (s - c.lo), snap_want(c, d2), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();  // published before any change of the row
  }
  __syncthreads();
}

// In-workgroup merge of one message (used when the receiver's row changed earlier in this
// sub-phase, so the precomputed classification may be stale).  Returns through *s_mod whether any
// record could change the row.
__device__ void merge_row_wg(const Ctx& c, uint32_t v, const Content& kc, int reason,
                             uint32_t phase, uint64_t* pend, uint32_t& npend, uint32_t* s_list, uint32_t* s_wave,
                             uint32_t* s_mod) {
  const uint32_t* __restrict__ rv = rec_row(c, v);
  const uint32_t n = c.n;
  __shared__ uint32_t s_pub;
  // one decision for the whole workgroup (threads reading the flag separately could disagree, and
  // the tile loop below branches around barriers on it)
  if (threadIdx.x == 0) s_pub = kc.snap && snap_published(kc) ? 1u : 0u;
  __syncthreads();
  const uint32_t* content = s_pub ? kc.snap : kc.live;
  __syncthreads();  // (s_pub is reused below)
  for (uint32_t base = 0; base < n; base += APPLY_TILE) {
    const uint32_t x0 = base + threadIdx.x * APPLY_CPT;
    uint32_t flags = 0;
    for (int pass = 0; pass < 2; ++pass) {
      flags = 0;
      for (int k = 0; k < APPLY_CPT; ++k) {
        const uint32_t x = x0 + k;
        if (x >= n) break;
        const uint32_t a = content[x];
        if (r_in_table(a) && sync_complex(a, rv[x], x == v)) flags |= 1u << k;
      }
      if (!kc.snap || content == kc.snap) break;
      // read from the live row: valid unless the sender published its copy meanwhile
      __threadfence();
      __syncthreads();
      if (threadIdx.x == 0) s_pub = snap_published(kc) ? 1u : 0u;
      __syncthreads();
      if (!s_pub) break;
      content = kc.snap;  // (uniform) the tile again, from the copy
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
        const uint32_t a = content == kc.snap ? kc.snap[x] : content_at(kc, x);
        if (update_membership(c, v, x, r_status(a), r_inc(a), reason, phase))
          pend[npend++] = ((uint64_t)x << 32) | (uint32_t)r_inc(a);
      }
    }
    __syncthreads();
  }
}

// one record row copied by the workgroup: 16-B accesses, 8 loads in flight per thread before the
// stores (a row is 4 x N bytes; one load-store round trip per word would take hundreds of us)
__device__ inline void copy_row(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t n) {
  if ((n & 3) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    const uint32_t n4 = n >> 2, step = blockDim.x * 8;
    for (uint32_t x0 = threadIdx.x; x0 < n4; x0 += step) {
      uint4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (x0 + j * blockDim.x < n4) v[j] = s4[x0 + j * blockDim.x];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (x0 + j * blockDim.x < n4) d4[x0 + j * blockDim.x] = v[j];
    }
  } else {
    for (uint32_t x = threadIdx.x; x < n; x += blockDim.x) dst[x] = src[x];
  }
}

// ---- the unsharded SYNC merge, classified in the receiver's workgroup (no classify launch).
// One message s -> r: (1) the block witness of both rows, chunk per thread — a 1,024-subject block
// where both rows equal the reference record (counts 0) holds identical records and is skipped
// unless it holds r's own subject as LEAVING (or, for the reverse direction, s's); (2) every other
// block streamed by the workgroup, 4 subjects per thread, both directions from one load: the forward
// complex records compacted in subject order and applied by thread 0 at once (each update touches
// only its own subject's cell, so classifying block j+1 after applying block j is exact), the
// reverse ones (the SYNC_ACK answering this SYNC merges r's row into s's: the same two rows) into the
// pool as rev_chunk / rev_total for the SYNC_ACK sub-phase and the lone-ack shortcut.  The content
// row is s's live row or its lazy snapshot (Content): the choice is made once for the workgroup and
// re-validated after every read of the live row.  s_need: LDS bitmask of the blocks to stream.
// prof: {blocks streamed, complex records, blocks}.
constexpr uint32_t NEED_WORDS = 512;  // (1 << 24 members) / 1,024 / 32
__device__ void sync_msg_wg(const Ctx& c, const Bufs& b, uint32_t r, uint32_t it, const SyncReq& rq, bool do_rev,
                            int reason, uint32_t phase, uint64_t* pend, uint32_t& npend, uint32_t* s_list,
                            uint32_t* s_wave, uint32_t* s_mod, uint32_t* s_need, uint32_t slot, bool& copied,
                            unsigned long long* prof) {
  __shared__ uint32_t s_pub3, s_rtot;
  const uint32_t n = c.n, chunks = b.chunks, tid = threadIdx.x, s = rq.from;
  const Content kc = msg_content(c, b, rq, 0);
  const uint32_t* bdv = c.bdiff + (size_t)(r - c.lo) * c.blocks;
  // the first chunk's witness words of both live rows and the self subjects' ref words, loaded beside
  // the content's slot lookup (a live word read before the snapshot flag is checked predates every
  // change of the sender's row; the receiver's row changes only in this workgroup)
  const uint32_t pc = tid < chunks ? c.bdiff[(size_t)(s - c.lo) * c.blocks + tid] : 0u;
  const uint32_t pv = tid < chunks ? bdv[tid] : 0u;
  const uint32_t rfr = c.ref[r], rfs = c.ref[s];
  if (tid == 0) {
    s_pub3 = kc.snap && snap_published(kc) ? 1u : 0u;
    s_rtot = 0;
  }
  for (uint32_t w = tid; w < (chunks + 31) / 32; w += blockDim.x) s_need[w] = 0;
  __syncthreads();
  bool from_snap = s_pub3 != 0;
  const uint32_t* rv = rec_row(c, r);
  const auto leaving = [](uint32_t rf) { return r_in_table(rf) && r_status(rf) == SWIM_LEAVING; };
  uint2* const rch = b.rev_chunk + (size_t)it * chunks;
  // (1) witness, chunk per thread
  for (int pass = 0; pass < 2; ++pass) {
    const uint32_t* bdc = from_snap ? kc.snap + n : c.bdiff + (size_t)(s - c.lo) * c.blocks;
    for (uint32_t ch = tid; ch < chunks; ch += blockDim.x) {
      const uint32_t base = ch * SYNC_CHUNK;
      const uint32_t wc = ch == tid && !from_snap ? pc : bdc[ch], wv = ch == tid ? pv : bdv[ch];
      const bool need = (wc | wv) != 0 || (r - base < (uint32_t)SYNC_CHUNK && leaving(rfr)) ||
                        (do_rev && s - base < (uint32_t)SYNC_CHUNK && leaving(rfs));
      if (need) atomicOr(&s_need[ch >> 5], 1u << (ch & 31));
      else if (do_rev) rch[ch] = make_uint2(0, 0);
    }
    if (!kc.snap || from_snap) break;
    __threadfence();  // the witness words are in before the flag is read again
    __syncthreads();
    if (tid == 0) s_pub3 = snap_published(kc) ? 1u : 0u;
    __syncthreads();
    if (!s_pub3) break;
    from_snap = true;  // s published its copy meanwhile: the witness again, from the copy
    for (uint32_t w = tid; w < (chunks + 31) / 32; w += blockDim.x) s_need[w] = 0;
    __syncthreads();
  }
  __syncthreads();
  // (2) the blocks to stream, in subject order
  uint32_t streamed = 0, cplx = 0;
  for (uint32_t w = 0; w < (chunks + 31) / 32; ++w) {
    uint32_t bits = s_need[w];
    while (bits) {
      const uint32_t ch = w * 32 + (uint32_t)__ffs(bits) - 1;
      bits &= bits - 1;
      ++streamed;
      const uint32_t base = ch * SYNC_CHUNK, x0 = base + 4 * tid;
      uint32_t flags = 0, rflags = 0;
      for (int pass = 0; pass < 2; ++pass) {
        const uint32_t* cr = from_snap ? kc.snap : kc.live;
        flags = rflags = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t x = x0 + q;
          if (x >= n || x0 >= base + SYNC_CHUNK) break;
          const uint32_t av = cr[x], ov = rv[x];
          if (r_in_table(av) && sync_complex(av, ov, x == r)) flags |= 1u << q;
          if (do_rev && r_in_table(ov) && sync_complex(ov, av, x == s)) rflags |= 1u << q;
        }
        if (!kc.snap || from_snap) break;
        __threadfence();
        __syncthreads();
        if (tid == 0) s_pub3 = snap_published(kc) ? 1u : 0u;
        __syncthreads();
        if (!s_pub3) break;
        from_snap = true;
      }
      // forward: compact in subject order, then thread 0 applies
      uint32_t total;
      const uint32_t off = block_exclusive_scan<APPLY_BLOCK>((uint32_t)__popc(flags), s_wave, &total);
      if (total) {
        uint32_t o = off;
        for (int q = 0; q < 4; ++q)
          if (flags & (1u << q)) s_list[o++] = x0 + q;
        if (!copied) {  // the first change of this row in the sub-phase: the lazy snapshot first
          lazy_snapshot(c, b, r, slot, 0);
          copied = true;
        }
        __syncthreads();
        if (tid == 0) {
          *s_mod = 1;
          for (uint32_t i = 0; i < total; ++i) {
            const uint32_t x = s_list[i];
            const uint32_t a = from_snap ? kc.snap[x] : content_at(kc, x);
            if (update_membership(c, r, x, r_status(a), r_inc(a), reason, phase))
              pend[npend++] = ((uint64_t)x << 32) | (uint32_t)r_inc(a);
          }
        }
        __syncthreads();
        cplx += total;
      }
      if (do_rev) {  // reverse: the subjects into the pool, in subject order
        uint32_t rt;
        const uint32_t roff = block_exclusive_scan<APPLY_BLOCK>((uint32_t)__popc(rflags), s_wave, &rt);
        if (tid == 0) {
          uint32_t pb = 0;
          if (rt) {
            pb = atomicAdd(&b.k->pool_cursor, rt);
            if (pb + rt > b.pool_cap) { set_err(c, ERR_PEND); rt = 0; }
          }
          s_list[0] = pb;
          s_list[1] = rt;
          rch[ch] = make_uint2(pb, rt);
          s_rtot += rt;
        }
        __syncthreads();
        const uint32_t pb = s_list[0], ok = s_list[1];
        if (ok) {
          uint32_t o = pb + roff;
          for (int q = 0; q < 4; ++q)
            if (rflags & (1u << q)) b.pool[o++] = x0 + q;
        }
        __syncthreads();
      }
    }
  }
  if (tid == 0) {
    if (do_rev) b.rev_total[it] = s_rtot;
    if (prof) {
      atomicAdd(prof, (unsigned long long)streamed);
      if (cplx) atomicAdd(prof + 1, (unsigned long long)cplx);
      atomicAdd(prof + 2, (unsigned long long)chunks);
    }
  }
  __syncthreads();
}

// canonical inbox order: deferred SYNC_ACKs (phantoms) first in their PAcks' creation order, then
// messages sent in earlier ticks (delayed), then (sender, ordinal / rank)
__device__ __forceinline__ uint64_t inbox_key(const Ctx& c, const SyncReq& q) {
  if (q.flags & RQ_PHANTOM) return q.pad;
  const uint32_t age = (q.flags & RQ_PARKED) ? min((uint32_t)c.T - q.pad, 2047u) : 0u;
  return (1ull << 63) | ((uint64_t)(2047u - age) << 52) | ((uint64_t)q.from << 24) | (q.ordinal & 0xffffffu);
}

// the receiver's inbox in canonical order (sending tick, sender, ordinal) -> s_it (item indices); its page table
// is reset for the next sub-phase.  Every thread of the workgroup calls it; returns the count.
// (inl0: the inbox's first inline slot, loaded by the caller with the receiver's other words)
__device__ inline uint32_t load_inbox(const Ctx& c, const Bufs& b, const SyInbox& x, uint32_t r, uint32_t k,
                                      uint32_t* s_it, uint64_t* s_key, uint32_t* s_raw, uint32_t inl0) {
  const uint32_t* inl = x.inl + (size_t)r * SY_INLINE;
  const uint32_t* tab = x.tab + (size_t)r * b.sy_max;
  if (k == 1) {  // the common inbox: nothing to order
    if (threadIdx.x == 0) s_it[0] = inl0;
    __syncthreads();
    return 1;
  }
  for (uint32_t q = threadIdx.x; q < k; q += blockDim.x) {
    uint32_t it;
    if (q < SY_INLINE) {
      it = inl[q];
    } else {
      const uint32_t pid = tab[(q - SY_INLINE) >> 6];
      it = pid < b.sy_pool_cap ? x.pool[(size_t)pid * 64 + ((q - SY_INLINE) & 63)] : NONE;
    }
    s_raw[q] = it;
    const SyncReq rq = x.items[it < b.req_cap ? it : 0];
    s_key[q] = it < b.req_cap ? inbox_key(c, rq) : ~0ull;  // unique per inbox
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < k; q += blockDim.x) {
    const uint64_t key = s_key[q];
    uint32_t rk = 0;
    for (uint32_t j = 0; j < k; ++j) rk += s_key[j] < key ? 1u : 0u;
    s_it[rk] = s_raw[q];
  }
  if (k > SY_INLINE)
    for (uint32_t pg = threadIdx.x; pg < (k - SY_INLINE + 63) / 64; pg += blockDim.x)
      x.tab[(size_t)r * b.sy_max + pg] = NONE;
  __syncthreads();
  return k;
}

// With message delay, between the SYNC and the SYNC_ACK sub-phases: each SYNC_ACK sent this tick draws
// its delay (the acker's SYNCACK_DELAY stream, keyed by the ack's inbox rank); a delayed one parks
// the acker's row as it is now (after its SYNC merges) and is deferred (RQ_DEFER: the SYNC_ACK
// sub-phase skips it).  One workgroup per ack; out of k_sync_apply, whose ack loop keeps its registers.
__global__ void __launch_bounds__(256) k_ack_delay(KP) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  __shared__ uint32_t s_slot;
  const uint32_t na = min(b.k->ack_total, b.req_cap);
  // this shard's acks: the local ones (items), then those bound for each other shard (tx_acks)
  uint32_t nt = na;
  if (c.xchg)
    for (uint32_t d = 0; d < c.world; ++d) nt += d == c.rank ? 0u : min(b.x->ack[d], b.tx_req_cap);
  for (uint32_t u = blockIdx.x; u < nt; u += gridDim.x) {
    SyncReq* ap;
    if (u < na) {
      ap = b.acks + u;
    } else {
      uint32_t k = u - na, d = 0;
      for (;; ++d) {
        if (d == c.rank) continue;
        const uint32_t m = min(b.x->ack[d], b.tx_req_cap);
        if (k < m) break;
        k -= m;
      }
      ap = b.tx_acks + (size_t)d * b.tx_req_cap + k;
    }
    SyncReq a = *ap;
    if (a.flags & (RQ_PARKED | RQ_DEFER)) continue;  // an arrival from the delay queue (uniform)
    const uint32_t dl = delay_ticks(c, a.from, a.to, a.from, SWIM_STREAM_SYNCACK_DELAY, a.ordinal, 0);
    if (!dl) {  // arrives now: a stopped receiver or its inbound filter drops it (skipped, as deferred)
      if (threadIdx.x == 0 && (!c.up[a.to] || !in_pass(c, a.to, a.from))) ap->flags = a.flags | RQ_DEFER;
      continue;
    }
    if (threadIdx.x == 0) s_slot = park_alloc(c, b);
    __syncthreads();
    const uint32_t slot = s_slot;
    if (slot != NONE) copy_row(rec_row(c, a.from), park_row(c, b, slot), c.n);
    __syncthreads();  // (the row is parked before the message is queued, and s_slot is reused)
    if (threadIdx.x == 0) {
      ap->flags = a.flags | RQ_DEFER;
      if (slot != NONE) {
        a.slot = 0;
        a.snap = slot;
        a.content = NONE;
        park_put(c, b, a, dl, true);
      }
    }
  }
}

// With message delay, before the SYNC sub-phase: (1) the content rows of this tick's delayed SYNCs
// (their senders' rows before any merge of the tick) into their park slots, one workgroup per row;
// (2) the delayed SYNCs and SYNC_ACKs arriving now into the inboxes (a message whose receiver stopped
// meanwhile is dropped); their slots are reusable from the next tick (k_end_tick).
__global__ void __launch_bounds__(256) k_sync_delay(KP) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  const uint32_t nj = min(b.k->park_jobs, b.park_cap);
  for (uint32_t j = blockIdx.x; j < nj; j += gridDim.x) {
    const uint2 jb = b.park_jobs[j];
    copy_row(rec_row(c, jb.y), park_row(c, b, jb.x), c.n);
  }
  const uint32_t bk = (uint32_t)T & DQ_MASK;
  const uint32_t cnt = min(b.sdq_cnt[bk], b.sdq_bcap);
  const SyncReq* dq = b.sdq + (size_t)bk * b.sdq_bcap;
  const uint32_t lane = threadIdx.x & 63;
  // (wave-uniform trip count: enqueue_sync's page discipline wants every lane of the wave)
  for (uint32_t i0 = blockIdx.x * blockDim.x + (threadIdx.x - lane); i0 < cnt; i0 += gridDim.x * blockDim.x) {
    const uint32_t i = i0 + lane;
    SyncReq q{};
    bool valid = i < cnt, ack = false;
    if (valid) {
      q = dq[i];
      ack = (q.flags & RQ_ACK) != 0;
      park_release(b, q.snap);
      valid = c.up[q.to] != 0;
      // the receiver stopped: the transport's send fails now — a start0 request's source completes
      // (an error resumes empty, MembershipProtocolImpl.java:268-276); its sender is owned here
      if (!valid && !ack && (q.flags & RQ_INITIAL) && c.up[q.from]) atomicAdd(&mem(c, q.from).init_done, 1u);
      valid = valid && in_pass(c, q.to, q.from);  // the receiver's inbound filter on arrival
      // an ack's receiver — and a SYNC's sender, whose ack may come back this tick — is merged into in
      // the SYNC_ACK sub-phase: if it is also read as SYNC_ACK content this tick (it received a SYNC),
      // it takes a snapshot slot (sflag_set_from; a receiver on another shard: k_recv_sync)
      const uint32_t who = ack ? q.to : q.from;
      if (valid && owned(c, who)) sflag_set(c, b, who - c.lo, SF_SENT);
      if (valid && !owned(c, q.to)) {  // into this tick's exchange (E2 / E3), content from the slot
        const uint32_t d = owner(c, q.to);
        const uint32_t j = atomicAdd(ack ? &b.x->ack[d] : &b.x->req[d], 1u);
        if (j < b.tx_req_cap) (ack ? b.tx_acks : b.tx_reqs)[(size_t)d * b.tx_req_cap + j] = q;
        else set_err(c, ERR_REQS);
        valid = false;
      }
    }
    enqueue_sync(c, b, 0, q, valid && !ack);
    enqueue_sync(c, b, 1, q, valid && ack);
  }
}

// D1 (d2 = 0): onSync at each receiver, then its SYNC_ACKs.  D2 (d2 = 1): the SYNC_ACK merge at
// the original senders (MembershipProtocolImpl.java:363-415).
// classified = 0 (SYNC_ACK sub-phase of an unsharded engine: no k_ack_classify launch): an ack takes
// the SYNC launch's reverse classification when its two rows are unchanged since (row_mod), and is
// classified in-workgroup (merge_row_wg) otherwise.
// fused = 1 (unsharded SYNC sub-phase): no k_sync_classify launch, every message is classified in
// the receiver's workgroup with the block witness (sync_msg_wg); prof as k_sync_classify's.
__device__ __forceinline__ void sync_apply_body(const Params* __restrict__ P, uint64_t T, int d2, int classified,
                                                int fused, unsigned long long* prof) {
  const Ctx c = pctx_sync(P, T);
  const Bufs b = P->b;
  __shared__ uint32_t s_need[NEED_WORDS];
  __shared__ uint32_t s_list[APPLY_TILE];
  __shared__ uint32_t s_wave[APPLY_BLOCK / 64 + 1];
  __shared__ uint32_t s_mod;
  __shared__ unsigned long long s_recs;
  __shared__ uint32_t s_iP[APPLY_BLOCK], s_iS[APPLY_BLOCK], s_iR[APPLY_BLOCK];
  __shared__ uint32_t s_it[SY_INBOX], s_raw[SY_INBOX];
  __shared__ uint64_t s_key[SY_INBOX];
  const SyInbox x = sy_inbox(b, d2);
  const uint2* const ichunk = d2 ? b.ack_chunk : b.item_chunk;
  const uint32_t* const itot = d2 ? b.ack_ctot : b.item_total;
  const uint32_t phase = d2 ? SWIM_PHASE_SYNCACK : SWIM_PHASE_SYNC;
  const uint32_t chunks = b.chunks;
  // the receiver list's entry is loaded beside its count (entries past the count are stale and
  // only read, never used)
  uint32_t s_spec = blockIdx.x < c.nl ? x.recv[blockIdx.x] : 0u;
  const uint32_t nrecv = *x.recv_cnt;
  uint64_t* pend = b.pend + (size_t)blockIdx.x * c.n;
  for (uint32_t ri = blockIdx.x; ri < nrecv; ri += gridDim.x) {
    const uint32_t s = s_spec;
    if (ri + gridDim.x < c.nl) s_spec = x.recv[ri + gridDim.x];
    // every word that depends on the receiver alone, in one batch
    const uint32_t li = s - c.lo;
    const uint32_t k = min(x.cnt[li], SY_INBOX);
    const uint32_t inl0 = x.inl[(size_t)li * SY_INLINE];
    const uint32_t tsz0 = mem(c, s).table_size, ins0 = mem(c, s).ins_rank;
    // start0's Flux still takes initial SYNC_ACKs (an answer after its completion or timeout is dropped)
    const bool iwait = d2 && mem(c, s).init_wait;
    // s both sent and received this tick (its roles are final since collection): other receivers
    // read this row as content while this workgroup merges into it, so it is copied into its slot
    // before the first change (lazy snapshot, Content above)
    const uint32_t slot = (d2 ? b.ack_snap : b.snap_idx)[li];
    bool copied = slot >= b.snap_cap;  // (no slot: nobody reads this row as content now)
    load_inbox(c, b, x, li, k, s_it, s_key, s_raw, inl0);
    if (threadIdx.x == 0) {
      mem(c, s).ev_minor = 0;
      mem(c, s).fetch_ctr = 0;
      s_mod = 0;
      s_recs = 0;
    }
    // the words the SYNC sub-phase's ack checks read for the first blockDim messages (up and inbound
    // filter of the ack's receiver, its sflag word) are loaded now, beside the merges' own loads, and
    // used after the merges (which change none of them); only without per-link settings / partition
    bool pre = false;
    uint8_t pre_up = 0, pre_in = 0;
    uint32_t pre_sf = 0;
    int32_t pre_loss = 0;
    if (!d2 && !c.n_links && !c.partition && threadIdx.x < k && s_it[threadIdx.x] < b.req_cap) {
      const uint32_t f = x.items[s_it[threadIdx.x]].from;
      pre = true;
      pre_loss = c.default_loss[s];
      pre_up = c.up[f];
      pre_in = c.default_inbound[f];
      pre_sf = owned(c, f) ? b.sflag[f - c.lo] : 0u;
    }
    __syncthreads();
    for (uint32_t q = 0; q < k; ++q) {
      const uint32_t it = s_it[q];
      if (it >= b.req_cap) continue;  // a page the pool could not give (ERR_REQS is set); uniform
      const SyncReq rq = x.items[it];
      if (d2 && ((rq.flags & RQ_DEFER) || ((rq.flags & RQ_INITIAL) && !iwait))) continue;  // (uniform)
      if (!d2 && (rq.flags & RQ_PHANTOM)) continue;  // a deferred SYNC_ACK: nothing to merge (uniform)
      const bool parked = (rq.flags & RQ_PARKED) != 0;
      const uint32_t tot_q = fused ? 0u : itot[it];  // issued with the header (stable since classify)
      const int reason = (d2 && (rq.flags & RQ_INITIAL)) ? R_INITIAL_SYNC : R_SYNC;
      // onSync's SYNC_ACK and start0's doFinally wait for the message's Monos (PAck): their waits are
      // collected while thread 0 merges it
      const bool waits = !d2 || reason == R_INITIAL_SYNC;
      if (waits && threadIdx.x == 0) wait_begin(c, s);
      uint32_t npend = 0;
      const uint32_t mod = s_mod;
      const bool own = d2 && !classified;  // this kernel classifies the ack
      uint32_t d1 = NONE;
      if (own && !parked && rq.pad != 0 && rq.content == NONE && b.row_mod[rq.from - c.lo] != (uint32_t)c.T &&
          b.row_mod[s - c.lo] != (uint32_t)c.T)
        d1 = rq.pad - 1;
      const bool pre = !fused && mod == 0 && (!own || d1 != NONE);  // precomputed classification is exact
      const uint32_t at = d1 != NONE ? d1 : it;
      const uint32_t tot = pre ? (d1 != NONE ? b.rev_total[at] : tot_q) : 0u;
      __syncthreads();  // every lane has read s_mod before lane 0 may set it
      if (fused && !parked) {  // unsharded SYNC sub-phase: the in-workgroup witness merge (no classify launch)
        sync_msg_wg(c, b, s, it, rq, CLS_REV && mod == 0, reason, phase, pend, npend, s_list, s_wave, &s_mod,
                    s_need, slot, copied, prof);
      } else if (!copied && (!pre || tot != 0)) {  // this message may change the row: the lazy snapshot first
        lazy_snapshot(c, b, s, slot, d2);
        copied = true;
      }
      if (fused && !parked) {
      } else if (pre) {  // the row is unchanged since classify
        if (threadIdx.x < 64 && tot != 0) {
          const Content kc = msg_content(c, b, rq, d2);
          // wave 0 reads the chunk results 64 at a time; lane 0 applies the non-empty chunks' complex
          // records in (chunk, subject) order
          const uint32_t lane = threadIdx.x;
          const uint2* ic = (d1 != NONE ? b.rev_chunk : ichunk) + (size_t)at * chunks;
          for (uint32_t c0 = 0; c0 < chunks; c0 += 64) {
            const uint2 e = c0 + lane < chunks ? ic[c0 + lane] : make_uint2(0, 0);
            uint64_t nz = __ballot(e.y != 0);
            while (nz) {
              const int j = __ffsll((unsigned long long)nz) - 1;
              nz &= nz - 1;
              const uint32_t base = __shfl(e.x, j, 64), cnt = __shfl(e.y, j, 64);
              if (lane == 0) {
                s_mod = 1;
                for (uint32_t q2 = 0; q2 < cnt; ++q2) {
                  const uint32_t xs = b.pool[base + q2];
                  const uint32_t a = content_at(kc, xs);
                  if (update_membership(c, s, xs, r_status(a), r_inc(a), reason, phase))
                    pend[npend++] = ((uint64_t)xs << 32) | (uint32_t)r_inc(a);
                }
              }
            }
          }
        }
      } else {
        merge_row_wg(c, s, msg_content(c, b, rq, d2), reason, phase, pend, npend, s_list, s_wave, &s_mod);
      }
      if (threadIdx.x == 0) {
        for (uint32_t j = 0; j < npend; ++j)
          apply_alive(c, s, (uint32_t)(pend[j] >> 32), (int32_t)(uint32_t)pend[j], reason, phase);
        s_recs += rq.flags >> RQ_RECS_SHIFT;
        if (!d2) {
          if (wait_end(c, s, rq.from, (rq.flags & RQ_INITIAL) ? PA_INITIAL_ACK : 0u))
            x.items[it].flags = rq.flags | RQ_WAIT;  // its SYNC_ACK waits
        } else if (waits) {
          wait_end(c, s, NONE, PA_INIT);
        }
      }
      __syncthreads();
    }
    if (!d2) {
      // the SYNC_ACKs, one thread per inbox message: the enqueues are independent (the receiver
      // orders its inbox), the loss draws keyed by the message's rank q
      const uint32_t tsz = s_mod ? mem(c, s).table_size : tsz0;  // (merges may have changed it)
      for (uint32_t q0 = 0; q0 < k; q0 += blockDim.x) {
        const uint32_t q = q0 + threadIdx.x;
        bool valid = false;
        SyncReq a{};
        if (q < k && s_it[q] < b.req_cap) {
          const uint32_t it = s_it[q];
          const SyncReq rq = x.items[it];
          const bool ph = (rq.flags & RQ_PHANTOM) != 0;
          const bool first = pre && q0 == 0;  // (pre_*: this message's words, loaded before the merges)
          const uint32_t t3 = (uint32_t)c.T << SF_BITS;
          const bool sf_now = first && (pre_sf & ~SF_MASK) == t3;
          // with message delay only the loss is decided now: the receiver's state and inbound filter
          // meet the ack when it arrives (k_ack_delay for an undelayed one, k_sync_delay else)
          // (a message whose Monos are still running sends its SYNC_ACK later, as a phantom)
          if (rq.flags & RQ_WAIT) {
          } else if (c.delay_on ? !lost_k(c, out_loss(c, s, rq.from), s, SWIM_STREAM_SYNCACK_OUT, q, 0)
              : first ? pre_up && !lost_k(c, pre_loss, s, SWIM_STREAM_SYNCACK_OUT, q, 0) && pre_in
                    : !out_fail(c, s, rq.from, s, SWIM_STREAM_SYNCACK_OUT, q, 0) && in_pass(c, rq.from, s)) {
            a.from = s; a.to = rq.from; a.ordinal = q; a.slot = 0;
            a.flags = RQ_DELIVERED | (rq.flags & RQ_INITIAL) | (tsz << RQ_RECS_SHIFT);
            a.content = NONE; a.snap = NONE;
            a.pad = CLS_REV && !ph && rq.content == NONE && !(rq.flags & RQ_PARKED) ? it + 1 : 0;
            valid = true;
            // the lone SYNC_ACK shortcut: the ack is the only one its receiver gets this tick (it sent
            // one SYNC and received none, so its row is unchanged since classify), this row did not
            // change in the SYNC merges, and the reverse classification of the pair found no record
            // that could change the receiver: its merge is a no-op, so the SYNC_ACK sub-phase's
            // bookkeeping for it (onSyncAck :385-391: the phase's minor / fetch counters restart, an
            // INITIAL ack completes a join step, the counters) is done here and nothing is enqueued
            if (valid && CLS_REV && !c.delay_on && !ph && rq.content == NONE && s_mod == 0 &&
                (first ? owned(c, rq.from) && !(sf_now && (pre_sf & SF_RECV)) &&
                             !(sf_now && (pre_sf & SF_MULTI))
                       : owned(c, rq.from) && !sflag_has(c, b, rq.from - c.lo, SF_RECV) &&
                             !sflag_has(c, b, rq.from - c.lo, SF_MULTI)) &&
                b.rev_total[it] == 0) {
              MemberDev& mf = mem(c, rq.from);
              mf.ev_minor = 0;
              mf.fetch_ctr = 0;
              if (rq.flags & RQ_INITIAL) mf.init_done += 1;
              stat_add(c, ST_SYNC_ACKS, 1);
              stat_add(c, ST_SYNC_RECORDS, tsz);
              valid = false;
            }
            if (valid && !owned(c, rq.from)) {  // content (this row after the SYNC merges) travels with the ack
              a.pad = 0;
              const uint32_t d = owner(c, rq.from);
              const uint32_t i = atomicAdd(&b.x->ack[d], 1u);
              if (i < b.tx_req_cap) b.tx_acks[(size_t)d * b.tx_req_cap + i] = a; else set_err(c, ERR_REQS);
              valid = false;
            }
          }
        }
        enqueue_sync(c, b, 1, a, valid);
      }
    }
    if (threadIdx.x == 0) {
      if (!d2) {
        if (s_mod) b.row_mod[s - c.lo] = (uint32_t)c.T;  // invalidates the reverse classifications
      } else {
        // start0's initial-sync completion counts the acks of its INITIAL SYNCs (:270-284)
        uint32_t init = 0, acks = 0;
        for (uint32_t q = 0; q < k; ++q) {
          if (s_it[q] >= b.req_cap) continue;
          const uint32_t fl = x.items[s_it[q]].flags;
          const bool ini = (fl & RQ_INITIAL) != 0;
          if ((fl & RQ_DEFER) || (ini && !iwait)) continue;  // skipped above
          init += ini ? 1u : 0u;
          acks++;
        }
        if (init) {
          mem(c, s).init_done += init;
          mem(c, s).init_last = (uint32_t)c.T;
        }
        stat_add(c, ST_SYNC_ACKS, acks);
      }
      x.cnt[s - c.lo] = 0;
      stat_add(c, ST_SYNC_RECORDS, s_recs);
    }
    __syncthreads();
    // this sub-phase's pingMembers inserts of s (its ADDED events, all made by this workgroup; none
    // when no merge changed the row and none were pending)
    if (s_mod || ins0) apply_ins_batch<APPLY_BLOCK, true>(c, s, threadIdx.x, s_iP, s_iS, s_iR);
  }
}

// the two sub-phases as two kernel symbols, so that a kernel trace times the SYNC merge (k_sync_apply)
// and the SYNC_ACK merge (k_ack_apply) separately, as the engine's HIP-event samples do
__global__ void __launch_bounds__(APPLY_BLOCK) k_sync_apply(KP, int classified, int fused, unsigned long long* prof) {
  sync_apply_body(P, T, 0, classified, fused, prof);
}
__global__ void __launch_bounds__(APPLY_BLOCK) k_ack_apply(KP, int classified) {
  sync_apply_body(P, T, 1, classified, 0, nullptr);
}
