// swim_quiet.h — the quiet fast path: many lockstep ticks in two launches while every member's work
// is provably member-local (DESIGN.md §5 "Quiet windows").  Included by swim_phases.h inside
// namespace swimdev, after the SYNC collection helpers.
//
// A cluster is QUIET at tick T when (checked on the device by k_quiet_scan):
//   * no live gossip at any up member, no pending failure-detector state (ack / relay timeouts, FD
//     SYNCs), no deferred list op, no join / leave / segmentation / compaction work pending;
//   * every up member's record row equals the reference row `ref` (block witness counts all zero,
//     DESIGN.md §5) and `ref` holds no SUSPECT or LEAVING record: every SYNC / SYNC_ACK merge is then
//     a no-op (identical records never change a row, MembershipRecord.isOverrides :67-88, and only
//     a LEAVING self record would re-run onSelfMemberDetected, MembershipProtocolImpl.java:604-607),
//     and a failure detector ALIVE result never differs from the view (onFailureDetectorEvent
//     :418-449 drops it);
//   * every up member holds the same table size (equal rows), so a SYNC carries the same record
//     count whoever sends it;
//   * no suspicion timer falls due (the wheel buckets of the window are empty);
// and the host has no control operation pending and no NetworkEmulator setting that a message's
// fate could depend on beyond the up / inbound-default words checked here (no loss, per-link
// setting, partition, delay, address route, recorded FD events: engine.hip quiet_eligible).
//
// Under these conditions a tick changes, per member, only the member's own scalars: doPing's period
// and cursor (FailureDetectorImpl.java:126-171; every ping is acknowledged at once), the gossip
// round's period++ with nothing to send (GossipProtocolImpl.java:143-151 returns before target
// selection), the periodic doSync's schedule and selectSyncAddress draws (MembershipProtocolImpl.java
// :339-357,461-472: the SYNC and its SYNC_ACK merge nothing), and the counters.  Members are then
// independent, and one thread can advance its member through a whole window of ticks: k_quiet_scan
// finds the first tick at which some member's step would leave this regime (a ping target that is
// down or inbound-blocked, a ping list that must be reshuffled, a due timer bucket) — the window
// ends there, and that tick runs on the per-tick kernel chain — and k_quiet_apply advances every
// member through the ticks before it.  The result is bit-for-bit the per-tick chain's
// (tests/test_quiet_path.py, tests/test_gpu_bench_parity.py).
#pragma once

struct QuietCtl {
  uint32_t fail;      // first tick offset (from T0) the window cannot cover (0xffffffff: none found)
  uint32_t tmin;      // min table size over up members (0xffffffff: none)
  uint32_t tmax_neg;  // 0xffffffff - max table size over up members
  uint32_t pad;
};

// the tick offset at which member v (up, owned) leaves the quiet regime within [T0, T0 + K), or K.
// Its pings of the window go to the next entries of its ping list (no reshuffle before the list's
// end); they are checked eight at a time: the list words in one batch of loads, then the targets'
// up / inbound words in another.  (cur, len, fdn, inbound: the member's words, loaded by the caller
// in its first batch)
constexpr uint32_t QUIET_BATCH = 8;
__device__ inline uint32_t quiet_member_scan(const Ctx& c, uint32_t v, uint64_t T0, uint32_t K, uint32_t cur,
                                             uint32_t len, uint32_t fdn, bool inbound, const uint32_t* fail,
                                             bool pingable) {
  const uint64_t Tend = T0 + K;
  if ((uint64_t)fdn >= Tend || fdn == NONE || len == 0) return K;  // no doPing, or period++ only
  const uint32_t np = (uint32_t)((Tend - 1 - fdn) / c.P) + 1;     // doPing calls in the window
  // the ping after the list's last entry reshuffles it (Collections.shuffle): the per-tick path
  uint32_t limit = np, end_off = K;
  if (cur + np > len) {
    limit = cur < len ? len - cur : 0u;
    end_off = (uint32_t)(fdn + (uint64_t)limit * c.P - T0);
  }
  // pingable: no member ever stopped or filtered its inbound traffic, so every target is up and
  // both inbound filters pass (only the reshuffle can end the window)
  if (pingable) return end_off;
  // the ping and its ack (tryFailOutbound on a stopped destination, both inbound filters); with no
  // loss and no delay this is the whole round trip
  if (limit && !inbound) return (uint32_t)(fdn - T0);
  const uint32_t* pl = ping_list(c, v) + cur;
  for (uint32_t k0 = 0; k0 < limit; k0 += QUIET_BATCH) {
    if (k0 && __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= (uint32_t)(fdn + (uint64_t)k0 * c.P - T0))
      return K;  // an earlier tick already ends the window
    uint32_t tg[QUIET_BATCH];
#pragma unroll
    for (uint32_t j = 0; j < QUIET_BATCH; ++j) tg[j] = k0 + j < limit ? pl[k0 + j] : v;
    uint32_t bad = 0;
#pragma unroll
    for (uint32_t j = 0; j < QUIET_BATCH; ++j) {
      const bool ok = c.up[tg[j]] != 0 && c.default_inbound[tg[j]] != 0;
      bad |= (k0 + j < limit && !ok) ? 1u << j : 0u;
    }
    if (bad) return (uint32_t)(fdn + (uint64_t)(k0 + __ffs(bad) - 1) * c.P - T0);
  }
  return end_off;
}

// One wait point for a batch of independent loads.  The compiler sinks a load into the branch that
// uses its value and waits for it there, so a batch written as one block of loads still ran as one
// round trip per branch; an empty asm that "modifies" every loaded value makes them all needed — and
// waited for — at one point, after all of them were issued.
#define QUIET_BATCH_WAIT(...) __asm__ volatile("" : __VA_ARGS__)
// a load through the global address space (global_load: waited for by vmcnt alone; a flat load —
// what a pointer read out of Ctx compiles to — also waits on lgkmcnt and returns out of order)
template <typename T>
__device__ __forceinline__ T gld(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
struct alignas(16) QU4 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ uint4 gld4(const void* p) {  // 16 B, 16-B aligned
  const __attribute__((address_space(1))) QU4* q = (const __attribute__((address_space(1))) QU4*)p;
  return make_uint4(q->x, q->y, q->z, q->w);  // (one dwordx4 load: the struct is 16-B aligned)
}

__device__ __forceinline__ void quiet_fail(uint32_t* fail, uint32_t off) {
  if (off < __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(fail, off);
}

// the words of MemberDev's first 48 B (the quiet check's and the quiet apply's): three 16-B loads
struct QuietMem {
  uint64_t ack_due, relay_due;
  uint32_t ping_cursor, ping_len, table_size, fd_sync_cnt, ins_rank;
  uint8_t join_now, join_pending, leave_pending, init_wait;
  uint64_t fd_period;
};
static_assert(sizeof(QuietMem) == 48 && offsetof(MemberDev, fd_period) == 40, "QuietMem mirrors MemberDev's head");
__device__ __forceinline__ QuietMem quiet_mem(const Ctx& c, uint32_t i) {
  const uint4* p = reinterpret_cast<const uint4*>(c.mem + i);
  uint4 w[3] = {p[0], p[1], p[2]};
  QuietMem m;
  __builtin_memcpy(&m, w, sizeof m);
  return m;
}

// k_quiet_scan: T = T0 (the window's first tick), K ticks.  Thread per owned member (grid-stride),
// plus the global checks spread over the grid: `ref` (every subject), the wheel buckets of the window.
// Every word a thread's first item needs — its ref word(s), its timer-bucket queue, the member's
// schedule, flags, witness count and MemberDev head — is loaded in ONE batch before any decision;
// the member's ping list and its targets' words follow (quiet_member_scan).  A thread's failing tick
// goes to the control block once, wave-reduced.
// Sharded engines: each shard's witness proves its rows equal ITS ref, so the shards' refs must be
// equal too (a partition healed after removal leaves each side's shard with its own ref): ref_a / ref_b
// are two arrays that agree at every subject iff they do — a local group passes shard 0's ref and
// this shard's, an RCCL engine the elementwise min and max of the ranks' refs (allreduced).
__global__ void __launch_bounds__(256) k_quiet_scan(KP, uint32_t K, QuietCtl* q, const uint32_t* ref_a,
                                                    const uint32_t* ref_b, uint32_t pingable) {
  const Ctx c = pctx(P, T);
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
  uint32_t* fail = &q->fail;
  const uint32_t W = c.wheel_mask + 1, nb = min(K, W), nwq = nb * c.wheel_nq;
  const uint32_t xmax = max(max(c.n, nwq), c.nl);
  uint32_t tmin = 0xffffffffu, tmax = 0, worst = K;
  for (uint32_t x = gtid; x < xmax; x += gsz) {
    // ---- one batch of independent loads
    const bool hs = x < c.n, hw = x < nwq, hm = x < c.nl;
    const uint32_t rf = hs ? c.ref[x] : 0u;
    const uint32_t ra = hs && ref_a ? ref_a[x] : 0u, rb = hs && ref_a ? ref_b[x] : 0u;
    uint32_t wj = 0, wc = 0;
    if (hw) {
      wj = x / c.wheel_nq;
      wc = c.wheel_cnt[(size_t)((T + wj) & c.wheel_mask) * c.wheel_nq + (x - wj * c.wheel_nq)];
    }
    const uint32_t v = c.lo + x;
    uint32_t mfl = 0, bz = 0, cf = 0, sf = 0, fdn = NONE;
    uint8_t upv = 0, inb = 0;
    GossipSched g{};
    QuietMem m{};
    if (hm) {
      mfl = c.mflag[x];
      upv = c.up[v];
      inb = c.default_inbound[v];
      bz = c.bnz[x];
      cf = c.compact_flag[x];
      sf = c.seg_flag[x];
      fdn = c.fd_next[x];
      g = c.gs[x];
      m = quiet_mem(c, x);
    }
    // ---- ref: no SUSPECT / LEAVING record in the table, and one ref for every shard
    if (hs && r_in_table(rf) && r_status(rf) != SWIM_ALIVE) worst = 0;
    if (hs && ref_a && ra != rb) worst = 0;
    // ---- suspicion timers due in the window (a queued entry may be a cancelled timer; the per-tick
    // path decides, so the window ends at the first non-empty bucket)
    if (hw && wc) worst = min(worst, wj);
    if (!hm) continue;
    if (mfl) { worst = 0; continue; }  // FD SYNCs / start0 / graceful stop / deferred SYNC_ACKs pending
    if (!upv) continue;
    // (an ack / relay deadline before T0 is a stale value of a member that was stopped: never due)
    // the record row equals ref: its block witness counts are all zero (the maintained count of
    // non-zero blocks, swim_device.h bdiff_add)
    const bool ok = g.len == 0 && cf == 0 && sf == 0 && m.ack_due < T && m.relay_due < T && m.fd_sync_cnt == 0 &&
                    m.ins_rank == 0 && !m.join_now && !m.join_pending && !m.leave_pending && !m.init_wait && bz == 0;
    if (!ok) { worst = 0; continue; }
    tmin = min(tmin, m.table_size);
    tmax = max(tmax, m.table_size);
    if (worst == 0) continue;
    worst = min(worst, quiet_member_scan(c, v, T, K, m.ping_cursor, m.ping_len, fdn, inb != 0, fail, pingable != 0));
  }
  // the wave's earliest failing tick and table sizes, one atomic each
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    tmin = min(tmin, (uint32_t)__shfl_xor(tmin, d, 64));
    tmax = max(tmax, (uint32_t)__shfl_xor(tmax, d, 64));
    worst = min(worst, (uint32_t)__shfl_xor(worst, d, 64));
  }
  // (each atomic only when it would change the word: with one table size everywhere, the first
  // waves set both words and the other ~1,000 skip them — same-address atomics serialise at the L2)
  if ((threadIdx.x & 63) == 0) {
    if (worst < K) quiet_fail(fail, worst);
    if (tmin != 0xffffffffu) {
      if (tmin < __hip_atomic_load(&q->tmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&q->tmin, tmin);
      const uint32_t tn = 0xffffffffu - tmax;
      if (tn < __hip_atomic_load(&q->tmax_neg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&q->tmax_neg, tn);
    }
  }
}

// the window the scan allowed (every shard's scan has completed: kernel boundary / collective)
__device__ __forceinline__ uint32_t quiet_window(const QuietCtl* q, uint32_t K) {
  const uint32_t tmin = q->tmin, tmax = 0xffffffffu - q->tmax_neg;
  return (tmin != 0xffffffffu && tmin != tmax) ? 0u : min(q->fail, K);
}

// doSync of up member v at tick t in a quiet window (sync_collect_fast / select_sync_address with the
// same draws); the receiver's merge and the SYNC_ACK's are no-ops, so what remains is the counters:
// ST_SYNCS for a selected target, the record counts of a delivered SYNC and its delivered ack
// (inb_v: v's inbound word, loaded by the caller.)  The first candidate is pure arithmetic (the
// draw), so what the common case decides on — its membership word in v's row, its up and inbound
// words — is loaded in ONE batch; a candidate that is not a member (a seed, or another draw: rare)
// takes the general path
// the first candidate of v's doSync at tick t (the draw: pure arithmetic)
__device__ __forceinline__ uint32_t quiet_sync_x0(const Ctx& c0, uint32_t v, uint64_t t) {
  Ctx c = c0;
  c.T = t;
  return next_int(draw(c, v, SWIM_STREAM_SYNC_SELECT, 0, 0), c.n);
}
// quiet_sync once the candidate's words are in (aw: its membership word in v's row, up0 / in0: its up
// and inbound words)
__device__ inline void quiet_sync_with(const Ctx& c0, uint32_t v, uint64_t t, uint32_t tsz, bool inb_v, uint32_t x0,
                                       uint32_t aw, uint32_t up0, uint32_t in0, unsigned long long& nsync,
                                       unsigned long long& nack, unsigned long long& nrec) {
  Ctx c = c0;
  c.T = t;
  uint32_t tg = x0;
  bool ok = up0 != 0 && in0 != 0;
  if (!(x0 != v && ((aw & A_IN_MEMBERS) || is_seed_of(c, v, x0)))) {
    tg = select_sync_address(c, v);
    if (tg == NONE) return;
    ok = c.up[tg] && c.default_inbound[tg];
  }
  // (branch-free counter updates: early returns here made the compiler keep the counters in scratch)
  nsync++;
  const unsigned long long dlv = ok ? 1ull : 0ull;           // delivered (else tryFailOutbound on a
                                                              // stopped target / inbound-blocked: dropped)
  const unsigned long long ack = ok && inb_v ? 1ull : 0ull;  // its SYNC_ACK passes v's inbound filter
  nack += ack;
  nrec += (dlv + ack) * tsz;  // onSync's syncMembership over the SYNC's records, onSyncAck's (:385-391)
}
__device__ inline void quiet_sync(const Ctx& c, uint32_t v, uint64_t t, uint32_t tsz, bool inb_v,
                                  unsigned long long& nsync, unsigned long long& nack, unsigned long long& nrec) {
  const uint32_t x0 = quiet_sync_x0(c, v, t);
  uint32_t aw = gld(aux_row(c, v) + x0), up0 = gld(c.up + x0), in0 = gld(c.default_inbound + x0);
  QUIET_BATCH_WAIT("+v"(aw), "+v"(up0), "+v"(in0));
  quiet_sync_with(c, v, t, tsz, inb_v, x0, aw, up0, in0, nsync, nack, nrec);
}

// The next window's scan, precomputed (QuietPre).  On a pristine cluster the scan's only per-window
// results are the first tick some member's ping list must be reshuffled and the first non-empty timer
// bucket; everything else it checks (flags, witness counts, ref, table sizes) no quiet window changes.
// So the apply that ends window k, whose threads hold every member's new schedule, also finds window
// k + 1's first failing tick for up to H ticks past its end, and window k + 1 — when nothing but
// windows ran in between (the host's pre_valid: every other API call and every per-tick tick clears
// it) — launches no scan.  The result is a tagged minimum, key = (~tag << 32) | offset, so a newer
// window's keys win over stale ones with no reset between windows; apply k's thread 0 writes the
// sentinel (tag, no failure) so that the tag is always present.
__device__ __forceinline__ uint64_t pre_key(uint32_t tag, uint32_t off) {
  return ((uint64_t)(0xffffffffu - tag) << 32) | off;
}

// k_quiet_apply: every owned member advanced through ticks [T, T + F), F = quiet_window(q) — or, when
// q is null, the window precomputed by the previous apply (pre_in, tag_in; a missing tag gives F = 0).
// `done` (pinned host memory) receives F; `next` is the other control block, reset here for the next
// scanned window (windows alternate between the two, so no copy precedes a scan).  H > 0: the next
// window is precomputed into pre_out under tag_out (pristine engines).  Thread 0 of workgroup 0 also
// performs the end-of-tick resets the skipped k_end_tick launches would have made (per-parity scratch
// counters, the witness rebase's dirty marks: with every up row equal to ref a rebase moves no
// reference record).
__global__ void __launch_bounds__(256) k_quiet_apply(KP, uint32_t K, const QuietCtl* q, QuietCtl* next,
                                                     uint32_t* done, uint32_t rebase_every, const uint64_t* pre_in,
                                                     uint32_t tag_in, uint64_t* pre_out, uint32_t tag_out,
                                                     uint32_t H) {
  const Ctx c = pctx(P, T);
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
  // ---- batch 1: the window's length and every word of the thread's first member (they do not
  // depend on the length: loaded beside it, one round trip where they took two)
  const bool own0 = gtid < c.nl;
  uint32_t upw = 0, inbw = 0, fdn = 0, sn0 = 0, gnext = 0, gper = 0, gw2 = 0, gw3 = 0;
  uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0, m6 = 0, m7 = 0, m8 = 0, m9 = 0, m10 = 0, m11 = 0;
  auto load_member = [&](uint32_t i) {
    const uint32_t v = c.lo + i;
    upw = gld(c.up + v), inbw = gld(c.default_inbound + v), fdn = gld(c.fd_next + i), sn0 = gld(c.sync_next + i);
    const uint4 gw4 = gld4(c.gs + i);
    const uint4* mp = reinterpret_cast<const uint4*>(c.mem + i);
    const uint4 w0 = gld4(mp), w1 = gld4(mp + 1), w2 = gld4(mp + 2);
    // (scalars for the asm operands: a vector component bound to an operand went through scratch)
    m0 = w0.x, m1 = w0.y, m2 = w0.z, m3 = w0.w, m4 = w1.x, m5 = w1.y, m6 = w1.z, m7 = w1.w, m8 = w2.x, m9 = w2.y,
    m10 = w2.z, m11 = w2.w;
    gnext = gw4.x, gper = gw4.y, gw2 = gw4.z, gw3 = gw4.w;
  };
  // (loaded unconditionally, a thread past the shard's end reading its last member: a load under a
  // branch is waited for inside it, where its value is copied to the join's register)
  load_member(c.nl ? min(gtid, c.nl - 1) : 0u);
  uint32_t qa = 0, qb = 0, qc = 0, kl = 0, kh = 0;
  if (q) {
    qa = gld(&q->tmin), qb = gld(&q->tmax_neg), qc = gld(&q->fail);
  } else {
    kl = gld(reinterpret_cast<const uint32_t*>(pre_in)), kh = gld(reinterpret_cast<const uint32_t*>(pre_in) + 1);
  }
  QUIET_BATCH_WAIT("+v"(upw), "+v"(inbw), "+v"(fdn), "+v"(sn0), "+v"(gnext), "+v"(gper), "+v"(m0), "+v"(m1),
                   "+v"(m2), "+v"(m3), "+v"(m4), "+v"(m5), "+v"(m6), "+v"(m7), "+v"(m8), "+v"(m9), "+v"(m10),
                   "+v"(m11), "+v"(qa), "+v"(qb), "+v"(qc), "+v"(kl), "+v"(kh));
  // quiet_window(q, K), or the window precomputed by the previous apply
  const uint32_t F = q ? ((qa != 0xffffffffu && qa != 0xffffffffu - qb) ? 0u : min(qc, K))
                       : (kh == 0xffffffffu - tag_in ? min(kl, K) : 0u);
  if (gtid == 0) {
    *done = F;
    *next = QuietCtl{0xffffffffu, 0xffffffffu, 0xffffffffu, 0u};
  }
  if (F == 0) return;
  const uint64_t Tend = T + F;
  uint32_t nfail = H;  // this thread's share of the next window's first failing offset (from Tend)
  // ---- batch 2: the next window's timer buckets (k_quiet_scan's check; four per thread a round) and
  // the first member's first doSync candidate words, waited for together
  const uint32_t W = c.wheel_mask + 1, nwq = H ? min(H, W) * c.wheel_nq : 0u;
  auto qaddr = [&](uint32_t x, uint32_t j) {
    return c.wheel_cnt + (size_t)((Tend + j) & c.wheel_mask) * c.wheel_nq + (x - j * c.wheel_nq);
  };
  // (every load unconditional, from a valid address whose value is then ignored where it does not
  // apply: see batch 1)
  const bool bq = gtid < nwq;
  const uint32_t nq1 = nwq ? nwq - 1 : 0u;
  const uint32_t xa = min(gtid, nq1), xb = min(gtid + gsz, nq1), xc = min(gtid + 2 * gsz, nq1), xd = min(gtid + 3 * gsz, nq1);
  const uint32_t ja = xa / c.wheel_nq, jb = xb / c.wheel_nq, jc = xc / c.wheel_nq, jd = xd / c.wheel_nq;
  uint32_t ca = gld(qaddr(xa, ja)), cb = gld(qaddr(xb, jb)), cc = gld(qaddr(xc, jc)), cd = gld(qaddr(xd, jd));
  const uint32_t v0 = c.lo + (c.nl ? min(gtid, c.nl - 1) : 0u);
  const bool sy = own0 && upw != 0 && sn0 != NONE && sn0 < Tend;
  const uint32_t sx = quiet_sync_x0(c, v0, sy ? sn0 : T);
  // (a member with no doSync in the window reads words of its own, already in the cache)
  uint32_t saw = gld(sy ? aux_row(c, v0) + sx : reinterpret_cast<const uint32_t*>(c.gs + (v0 - c.lo))),
           sup = gld(c.up + (sy ? sx : v0)), sin = gld(c.default_inbound + (sy ? sx : v0));
  QUIET_BATCH_WAIT("+v"(ca), "+v"(cb), "+v"(cc), "+v"(cd), "+v"(saw), "+v"(sup), "+v"(sin));
  if (H) {
    if (gtid == 0) atomicMin(reinterpret_cast<unsigned long long*>(pre_out), pre_key(tag_out, 0xffffffffu));
    if (bq) {
      if (ca) nfail = min(nfail, ja);
      if (cb && gtid + gsz < nwq) nfail = min(nfail, jb);
      if (cc && gtid + 2 * gsz < nwq) nfail = min(nfail, jc);
      if (cd && gtid + 3 * gsz < nwq) nfail = min(nfail, jd);
    }
    // further rounds (more bucket queues than four per thread: long precomputed windows)
    for (uint32_t x0 = gtid + 4 * gsz; x0 < nwq; x0 += 4 * gsz) {
      const uint32_t xa = x0, xb = min(x0 + gsz, nwq - 1), xc = min(x0 + 2 * gsz, nwq - 1), xd = min(x0 + 3 * gsz, nwq - 1);
      const uint32_t ka = xa / c.wheel_nq, kb = xb / c.wheel_nq, kc = xc / c.wheel_nq, kd = xd / c.wheel_nq;
      uint32_t da = *qaddr(xa, ka), db = *qaddr(xb, kb), dc = *qaddr(xc, kc), dd = *qaddr(xd, kd);
      QUIET_BATCH_WAIT("+v"(da), "+v"(db), "+v"(dc), "+v"(dd));
      if (da) nfail = min(nfail, ka);
      if (db && x0 + gsz < nwq) nfail = min(nfail, kb);
      if (dc && x0 + 2 * gsz < nwq) nfail = min(nfail, kc);
      if (dd && x0 + 3 * gsz < nwq) nfail = min(nfail, kd);
    }
  }
  if (gtid == 0) {
    const Bufs& b = P->b;
    b.snap_cnt[0] = b.snap_cnt[1] = 0;
    c.gclaim_cnt[0] = c.gclaim_cnt[1] = 0;
  }
  const uint64_t first_rebase = (T + rebase_every - 1) / rebase_every * rebase_every;
  if (first_rebase < Tend)
    for (uint32_t s = gtid; s < c.n; s += gsz) c.dirty[s] = 0u;
  unsigned long long npings = 0, nsync = 0, nack = 0, nrec = 0;
  for (uint32_t i = gtid; i < c.nl; i += gsz) {
    const uint32_t v = c.lo + i;
    const bool first = i == gtid;
    if (!first) {  // (a grid smaller than the shard: every word in one batch, waited for once)
      load_member(i);
      QUIET_BATCH_WAIT("+v"(upw), "+v"(inbw), "+v"(fdn), "+v"(sn0), "+v"(gnext), "+v"(gper), "+v"(m0), "+v"(m1),
                       "+v"(m2), "+v"(m3), "+v"(m4), "+v"(m5), "+v"(m6), "+v"(m7), "+v"(m8), "+v"(m9), "+v"(m10),
                       "+v"(m11));
    }
    const bool up = upw != 0, inb = inbw != 0;
    const GossipSched g{gnext, gper, gw2, gw3};
    QuietMem qm;  // (field by field from the words: a memcpy of a uint4 array put it in scratch)
    qm.ack_due = (uint64_t)m1 << 32 | m0;
    qm.relay_due = (uint64_t)m3 << 32 | m2;
    qm.ping_cursor = m4;
    qm.ping_len = m5;
    qm.table_size = m6;
    qm.fd_sync_cnt = m7;
    qm.ins_rank = m8;
    qm.join_now = (uint8_t)m9;
    qm.join_pending = (uint8_t)(m9 >> 8);
    qm.leave_pending = (uint8_t)(m9 >> 16);
    qm.init_wait = (uint8_t)(m9 >> 24);
    qm.fd_period = (uint64_t)m11 << 32 | m10;
    MemberDev& m = c.mem[i];
    // ---- FD (doPing every pingInterval; acknowledged at once)
    if (up && fdn < Tend) {
      const uint32_t k = (uint32_t)((Tend - 1 - fdn) / c.P) + 1;
      m.fd_period = qm.fd_period + k;
      m.ev_minor = 0;
      if (qm.ping_len) {
        m.ping_cursor = qm.ping_cursor + k;
        npings += k;
      }
      c.fd_next[i] = fdn + k * c.P;
    }
    // ---- gossip rounds (the timer runs while down; period++ only while up)
    if (g.next < Tend) {
      const uint32_t r = (uint32_t)((Tend - 1 - g.next) / c.G) + 1;
      GossipSched& gw = c.gs[i];
      gw.next = g.next + r * c.G;
      if (up) gw.period = g.period + r;
    }
    // ---- periodic SYNC (the schedule advances while down too, sync_collect_fast); the first one's
    // candidate words came with batch 2
    uint32_t sn = sn0;
    if (sn != NONE && sn < Tend) {
      if (first && sy) {
        quiet_sync_with(c, v, sn, qm.table_size, inb, sx, saw, sup, sin, nsync, nack, nrec);
        sn += c.S;
      }
      for (; sn < Tend; sn += c.S)
        if (up) quiet_sync(c, v, sn, qm.table_size, inb, nsync, nack, nrec);
      c.sync_next[i] = sn;
    }
    // ---- the next window (quiet_member_scan with every target pingable): the member's ping list
    // reaches its end — the ping that would reshuffle it
    if (H && up) {
      const uint32_t fdn1 = fdn < Tend ? fdn + ((uint32_t)((Tend - 1 - fdn) / c.P) + 1) * c.P : fdn;
      const uint32_t cur1 = fdn < Tend && qm.ping_len ? qm.ping_cursor + (uint32_t)((Tend - 1 - fdn) / c.P) + 1
                                                      : qm.ping_cursor;
      nfail = min(nfail, quiet_member_scan(c, v, Tend, H, cur1, qm.ping_len, fdn1, true, nullptr, true));
    }
  }
  if (H) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) nfail = min(nfail, (uint32_t)__shfl_xor(nfail, d, 64));
    if ((threadIdx.x & 63) == 0 && nfail < H)
      atomicMin(reinterpret_cast<unsigned long long*>(pre_out), pre_key(tag_out, nfail));
  }
  wave_stat_add(c, ST_PINGS, npings);
  wave_stat_add(c, ST_FD_EVENTS, npings);  // publishPingResult(ALIVE) per acknowledged ping
  wave_stat_add(c, ST_SYNCS, nsync);
  wave_stat_add(c, ST_SYNC_ACKS, nack);
  wave_stat_add(c, ST_SYNC_RECORDS, nrec);
}
