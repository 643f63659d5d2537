"""Headline benchmark: simulated member-protocol-periods/sec at N=65,536 (BASELINE.json `metric`).

One step = one SWIM protocol period (ping_interval of virtual time: 10 ticks of 100 ms with the LAN
defaults) for all N members: FD pings / ping-reqs, 5 gossip rounds, staggered periodic SYNC
(N/300 full-table exchanges per tick), suspicion timers and event compaction — the whole hot path of
SURVEY.md §8 on synthetic input (the headline: a converged N-member cluster with no faults; the
failures workload kills a member every 20 periods; the churn workload is BASELINE config 3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--members 65536] [--workload quiet|failures|churn]

The engine advances a provably quiet cluster through whole windows of ticks with two kernel launches
(swim_quiet.h, DESIGN.md §5: every member's tick is member-local, bit-exact with the per-tick kernel
chain), and the per-tick chain for every tick that needs it.  With N > 1 (`--gpus N` starts
torch.distributed.run with N ranks itself, as a child process; or the driver launches it) the SAME
N-member cluster is row-sharded over the N GPUs (swim_create_shard): each rank owns members
[r*N/G, (r+1)*N/G), cross-shard GOSSIP_REQ / SYNC / SYNC_ACK traffic is pulled by device kernels from
the producers' exchange regions over xGMI, counts by ncclAllToAll inside the library.
Total work is fixed, so `scaling` is "strong".  torch.distributed (gloo) only bootstraps RCCL and
brackets the timed region with barriers.

Prints ONE JSON line with `value` (whole-job member-periods/s) and the rooflines of the kernels that
carried the step (`roofline`: the quiet windows' k_quiet_scan + k_quiet_apply; `roofline_step`: the
whole step against its wall time), plus — single GPU, quiet workload — side runs on the same N: the
per-tick kernel chain (`per_tick_path`, with the SYNC merge's roofline), the failures workload
(`failures`, with the fanout and delivery kernels' rooflines), BASELINE config 3 (`churn`, N =
16,384), the KS timing mode (`ks_mode`), and the CPU oracle on the box's cores (`cpu_baseline`).
Every kernel time is HIP events on the engine's own stream.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md: 8.0 TB/s)
KILL_EVERY = 20
KILL_FIRST = 10
CHURN_PER_MILLE = 10    # config 3: 1 % of the members killed and as many fresh members joined per period
CHURN_LOSS = 5          # config 3: 5 % uniform outbound loss


WORKLOAD = "quiet"
LAN = "LAN defaults (ping 1 s / gossip 200 ms / sync 30 s staggered)"
WORKLOAD_TEXT = {
    "quiet": "config4-lan-quiet: N={n} members (one cluster), " + LAN + ", 0% loss, no faults",
    "failures": "config4-lan-failures: N={n} members (one cluster), " + LAN + ", 0% loss, "
                "one member killed every {every} periods",
    "churn": "config3-churn: N={n} live members, " + LAN + ", {loss}% uniform outbound loss, {churn} kills + "
             "{churn} fresh joins via seed 0 per period",
}
DEFAULT_MEMBERS = {"quiet": 65536, "failures": 65536, "churn": 16384}


class Schedule:
    """The workload's control operations, applied at the start of each period (identical on every
    rank: the control state they change is replicated).
      quiet     nothing (BASELINE config 4 at 0 % loss);
      failures  one member killed every KILL_EVERY periods;
      churn     BASELINE config 3: 5 % uniform loss, and every period 1 % of the members killed
                and as many fresh members joined through seed member 0."""

    def __init__(self, workload, n, periods, churn=None, loss=None):
        import random
        self.workload, self.n = workload, n
        self.loss = CHURN_LOSS if loss is None else loss
        self.churn = (churn if churn is not None else max(1, n * CHURN_PER_MILLE // 1000)) if workload == "churn" else 0
        self.capacity = n + self.churn * periods
        self.live = list(range(1, n))  # member 0 is the seed and stays up
        self.next_id = n
        self.rng = random.Random(12345)
        self.progress = False  # --progress: a stderr line per step (long churn runs)

    def setup(self, e):
        if self.workload == "churn":
            e.set_default_loss(self.loss)
            e.set_seeds([0])

    def ops(self, p):
        if self.workload == "failures":
            if p >= KILL_FIRST and (p - KILL_FIRST) % KILL_EVERY == 0:
                return [("kill", (17 + 7919 * ((p - KILL_FIRST) // KILL_EVERY)) % self.n)]
            return []
        if self.workload == "churn":
            out = []
            for _ in range(self.churn):
                out.append(("kill", self.live.pop(self.rng.randrange(len(self.live)))))
            for _ in range(self.churn):
                out.append(("join", self.next_id))
                self.live.append(self.next_id)
                self.next_id += 1
            return out
        return []

    def run(self, e, p0, p1):
        """Advance e through periods [p0, p1), one step per run of op-free periods."""
        p = p0
        while p < p1:
            for op, m in self.ops(p):
                getattr(e, op)(m)
            nxt = p + 1
            while nxt < p1 and not self._has_ops(nxt):
                nxt += 1
            e.step(nxt - p)
            p = nxt
            if self.progress:
                st = e.stats()
                print(f"bench: period {p}/{p1} t={time.time():.3f} gossips={st['gossips_created']} "
                      f"msgs={st['gossip_messages']} syncs={st['syncs']}", file=sys.stderr, flush=True)

    def _has_ops(self, p):
        if self.workload == "failures":
            return p >= KILL_FIRST and (p - KILL_FIRST) % KILL_EVERY == 0
        return self.workload == "churn"


def make_config(lib, device=0):
    from swimgpu import abi
    return abi.default_config(lib, 0, sync_stagger=1, record_fd_events=0, device=device)


def churn_capacities(cfg, capacity):
    """Config-3 churn sizes (also used by tests/test_gpu_configs.py).  A period's joins add every
    joiner at every viewer (millions of events); every member holds every gossip of the last
    periodsToSweep periods, and every member that learns news through SYNC gossips it (DESIGN.md §6:
    the live gossips per member grow by ~8 x N per period); a period's kills put a suspicion timer
    at every viewer within a few seconds."""
    cfg.event_capacity = 1 << 25
    cfg.gossip_capacity = 1 << 18  # 24 B per (member, gossip): 103 GB of slab at N = 16,384
    # one gossip round's GOSSIP_REQs: ~4 x 10^8 in the third period at N = 16,384
    cfg.message_capacity = 1 << 30 if capacity > 12288 else 1 << 28
    # a viewer keeps a SequenceIdCollector per gossiper heard until it is removed
    cfg.collector_capacity = 1 << (2 * capacity - 1).bit_length()
    # 5 % loss drops gossips, so collectors fragment (many spilled interval blocks), and every
    # false suspicion puts a timer at every viewer
    cfg.interval_capacity = 8192
    cfg.timer_capacity = 64 * capacity
    # pending at once: a period's kills (and false suspicions) at every viewer, for the suspicion
    # timeout (5 x ceil_log2(N) periods): ~2.2 x 10^8 at N = 16,384
    cfg.timer_pool_capacity = 1 << 28 if capacity > 12288 else 1 << 27
    return cfg


def build_hash():
    """The source hash of the libswimgpu.so build (the stamp __graft_entry__.build writes beside it):
    a profile is attached to this run only if it measured the same build."""
    try:
        return open(os.path.join(REPO, "scalecube-cluster_amd", "lib", "libswimgpu.so.srchash")).read().strip()[:16]
    except OSError:
        return None


def bench_key(args, n):
    """What identifies this command's kernel launches: every argument that changes what the engines
    run (tools/prof_summary.py stores the profiled command's key; a profile is used only by a run
    with the same key and build)."""
    return {"gpus": args.gpus, "steps": args.steps, "warmup": args.warmup, "workload": args.workload,
            "members": n, "local_shards": args.local_shards, "extras": not args.no_extras,
            "churn": not args.no_churn, "fanout_steps": args.fanout_steps, "churn_steps": args.churn_steps}


_PROFILE = {}


def find_profile(key):
    """The newest committed per-launch PMC profile (profiles/*_pmc.json, tools/prof_driver.sh ->
    tools/prof_summary.py) of THIS command on THIS build: (doc, path) or (None, reason).  Never picked
    by file name order: a profile of another build or another command is not used."""
    ck = json.dumps(key, sort_keys=True)
    if ck in _PROFILE:
        return _PROFILE[ck]
    import glob
    bh, best, seen = build_hash(), None, 0
    for path in glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if "engines" not in d:
            continue
        seen += 1
        if d.get("build") != bh or d.get("bench_key") != key:
            continue
        if best is None or d.get("created", "") > best[0].get("created", ""):
            best = (d, os.path.relpath(path, REPO))
    _PROFILE[ck] = best or (None, f"none of the {seen} per-launch PMC profiles under profiles/ measured this "
                                  f"command on this build ({bh})")
    return _PROFILE[ck]


def profile_launches(doc, engine, kernel, first=None, last=None):
    """Per-launch HBM bytes (and kernel-trace microseconds) of `kernel` in the profiled command's
    `engine`-th engine (engines in creation order): the launch #first, or the mean of the last `last`
    launches.  None if the profile does not hold them."""
    engs = doc.get("engines") or []
    if engine >= len(engs):
        return None
    k = engs[engine].get(kernel)
    if not k:
        return None
    hb, fb, wb, us = k["hbm_bytes"], k["fetch_bytes"], k["write_bytes"], k.get("us") or []
    if first is not None:
        if first >= len(hb):
            return None
        pick = [first]
        tpick = pick if first < len(us) else None  # (launch #first of the trace pass: same program order)
    else:
        if not last or len(hb) < last:
            return None
        pick = list(range(len(hb) - last, len(hb)))
        tpick = pick if len(us) == len(hb) else None
    mean = lambda xs, ix: sum(xs[i] for i in ix) / len(ix) if ix else None
    return {"hbm": mean(hb, pick), "fetch": mean(fb, pick), "write": mean(wb, pick), "us": mean(us, tpick),
            "launches": len(pick)}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def side_run(lib, workload, n, warmup, steps, device=0, quiet=True, period_times=None, **knobs):
    """A secondary single-GPU measurement on its own engine (the headline engine is closed first):
    `warmup` untimed periods, then `steps` timed ones.  Returns (seconds, merge profile, fanout
    profile, stats, deliver profile, quiet-window stats).  period_times (a list): each timed period's
    seconds are appended (a synchronisation after each; for workloads whose periods take seconds)."""
    import torch
    from swimgpu import abi
    sch = Schedule(workload, n, warmup + steps)
    cfg = make_config(lib, device)
    if workload == "churn":
        churn_capacities(cfg, sch.capacity)
    for k, v in knobs.items():
        setattr(cfg, k, v)
    e = abi.Engine(lib, cfg, sch.capacity, n, 1)
    try:
        e.set_quiet_path(quiet)
        sch.setup(e)
        sch.run(e, 0, warmup)
        e.drain_events()
        torch.cuda.synchronize()
        e.profile_enable(True)
        q0 = e.quiet_stats()
        t0 = time.perf_counter()
        if period_times is None:
            sch.run(e, warmup, warmup + steps)
        else:
            for p in range(warmup, warmup + steps):
                tp = time.perf_counter()
                sch.run(e, p, p + 1)
                torch.cuda.synchronize()
                period_times.append(time.perf_counter() - tp)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        q1 = e.quiet_stats()
        out = (dt, e.profile_merge(), e.profile_fanout(), e.stats(), e.profile_deliver(),
               {k: q1[k] - q0[k] for k in q1})
        e.drain_events()
    finally:
        e.close()
    return out


def window_pmc_traffic(key, scanned=True, first=None):
    """HBM bytes of the timed quiet window (k_quiet_apply, plus k_quiet_scan when the window's end was
    not precomputed) from the per-launch PMC profile of this exact command and build: the launch
    #first[kernel] of the main engine (the launches before it are the warm-up's).  (None, reason)
    otherwise: traffic is never borrowed from another window, command or build."""
    doc, src = find_profile(key)
    if doc is None:
        return None, src, None
    tot, us = 0.0, 0.0
    for k in (("k_quiet_scan", "k_quiet_apply") if scanned else ("k_quiet_apply",)):
        pl = profile_launches(doc, 0, k, first=first.get(k, 0))
        if pl is None:
            return None, f"{src} holds no launch #{first.get(k, 0)} of {k}", None
        tot += pl["hbm"]
        us = None if us is None or pl["us"] is None else us + pl["us"]
    return tot, src, us


def timed_launch_index(qs0, local_shards=1):
    """The timed window's launch of each quiet kernel in the profiled command (0-based): the warm-up's
    launches come first — k_quiet_apply once per window ATTEMPT (an attempt that advances no tick
    launches it too), k_quiet_scan once per attempt whose end was not precomputed, each once per
    local shard (swim_quiet_stats counted before the timed region)."""
    sh = max(1, local_shards)
    return {"k_quiet_apply": qs0["attempts"] * sh, "k_quiet_scan": (qs0["attempts"] - qs0.get("precomputed", 0)) * sh}


def hbm_fields(traffic, seconds):
    """the real HBM rate beside the rule-based one: the profiled bytes of the launch over its HIP-event time"""
    if traffic is None or not seconds:
        return {"hbm_achieved": None, "hbm_frac": None}
    a = traffic / seconds / 1e9
    return {"hbm_achieved": a, "hbm_frac": a / HBM_PEAK_GBPS}


def quiet_roofline(qprof, key, scanned=True, first=None):
    """k_quiet_apply (+ k_quiet_scan when the window's end was not precomputed) of the timed window
    against HBM, two ways: `frac` by SURVEY.md §8(d)'s rule — swim_profile_quiet's algorithmic bytes
    (21 B per member-period of the ping phase, plus the quiet check's reads once per window) over the
    kernels' HIP-event time — which credits per-period bytes the closed form does not move (it
    advances a member's cursor and period in O(1)), so it grows with the window's length; and
    `hbm_frac`, the bytes the timed launch really moved (per-launch PMC of this exact command and
    build, window_pmc_traffic) over the same time."""
    per_win = qprof["alg_bytes"] / max(1, qprof["launches"])
    secs = qprof["total_ms"] / max(1, qprof["launches"]) / 1e3
    ach = qprof["alg_bytes"] / max(1e-12, qprof["total_ms"] / 1e3) / 1e9
    traffic, src, prof_us = window_pmc_traffic(key, scanned, first) if qprof["launches"] == 1 else \
        (None, "more than one window in the timed region", None)
    kern = ("k_quiet_scan + k_quiet_apply (one quiet window)" if scanned else
            "k_quiet_apply (one quiet window, its end precomputed by the window before: no scan)")
    return {"bound": "hbm", "kernel": kern, "achieved": ach,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS, "traffic": traffic,
            **hbm_fields(traffic, secs),
            "traffic_unit": "HBM bytes of the timed window's launch (rocprofv3 memory-side read / write requests "
                            "x their sizes, tools/prof_summary.py; this command, this build)",
            "traffic_source": src, "profiled_launch_us": prof_us,
            "windows": qprof["launches"], "avg_window_ms": secs * 1e3,
            "alg_bytes_per_window": per_win, "ticks_per_window": qprof["messages"] / max(1, qprof["launches"]),
            "member_periods_per_window": qprof["records"] / max(1, qprof["launches"]),
            "alg_bytes_rule": "21 B per member-period (SURVEY.md §8(d) ping phase) + per window the quiet check's "
                              "reads: the 4-B count of non-zero witness blocks + 64 B of member words per row, "
                              "4 B per subject of the reference row, 4 B per timer-bucket queue (swim.h "
                              "swim_profile_quiet)"}


def steady_state(e, sch, args, n, cold_dt, barrier, se=None, calls=7):
    """The headline repeated: `calls` further swim_step calls of the same length right after the timed
    one (each bracketed by the same barrier + synchronisation), so the line carries the steady-state
    rate beside the driver's single timed call.  `value` stays the driver's definition (the one
    call); the first call after the warm-up pays more (cold_call_penalty_us)."""
    import statistics
    p, ts = args.warmup + args.steps, []
    for _ in range(calls):
        barrier()
        t0 = time.perf_counter()
        sch.run(e, p, p + args.steps)
        barrier()
        dt = time.perf_counter() - t0
        ts.append(se.max_time(dt) if se is not None else dt)
        p += args.steps
    med = statistics.median(ts)
    return {"calls": calls, "periods_per_call": args.steps, "call_us": [round(t * 1e6, 2) for t in ts],
            "median_call_us": med * 1e6, "value": n * args.steps / med, "unit": "member-periods/s",
            "ms_per_step": med / args.steps * 1e3, "cold_call_us": cold_dt * 1e6,
            "cold_call_penalty_us": (cold_dt - med) * 1e6,
            "note": "median of identical swim_step calls after the timed one (same length, barrier + synchronize "
                    "around each); `value` above is the first (cold) call, as the driver defines it"}


def quiet_window_model(e, n, tpp, lengths=(1, 4, 20, 100), budget_s=3.0):
    """How the headline depends on how far one swim_step call advances (after the timed region, on
    the same engine): for calls of L periods each, the quiet window's GPU time (HIP events) and the
    wall time per call; a least-squares fit window_us = fixed + per_tick x ticks gives the fixed cost
    of a window and the marginal member-periods/s of its length-proportional part.  `one_period_step`
    is the rate a caller sees that advances one period per call (the Java shim's
    SimulatedCluster.advance)."""
    import torch
    pts = []
    for L in lengths:
        reps = max(2, min(50, int(200 // L)))
        e.profile_enable(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        done = 0
        for _ in range(reps):
            e.step(L)
            done += 1
            if time.perf_counter() - t0 > budget_s:
                break
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / done
        q = e.profile_quiet()
        pts.append({"periods_per_call": L, "ticks_per_call": L * tpp, "calls": done,
                    "windows": q["launches"], "window_us": q["total_ms"] * 1e3 / max(1, q["launches"]),
                    "call_us": wall * 1e6, "member_periods_per_s": n * L / wall})
    import numpy as np
    xs = np.array([p["ticks_per_call"] for p in pts], dtype=float)
    ys = np.array([p["window_us"] for p in pts], dtype=float)
    cs = np.array([p["call_us"] for p in pts], dtype=float)
    slope, fixed = np.polyfit(xs, ys, 1)
    cslope, cfixed = np.polyfit(xs, cs, 1)
    e.profile_enable(False)
    return {"points": pts, "fixed_us_per_window": float(fixed), "us_per_tick": float(slope),
            "marginal_member_periods_per_s": float(n / (slope * tpp) * 1e6) if slope > 0 else None,
            "fixed_us_per_call": float(cfixed),
            "one_period_step": pts[0]["member_periods_per_s"],
            "note": "value = N x periods / wall time of ONE swim_step call over the timed periods: it rises with "
                    "the periods per call (fixed_us_per_call is paid once per call); see points"}


def merge_roofline(prof, world, local_shards, dt, steps, tpp, key=None, engine=None):
    """The SYNC merge: k_sync_apply's SYNC launch (unsharded: classification fused) or k_sync_classify
    (sharded), HIP events on one launch in three; traffic = the mean of the timed periods' launches
    in the per-launch PMC profile of this command and build (engine = the run's engine index)."""
    merge_kernel = "k_sync_apply" if world == 1 and local_shards == 1 else "k_sync_classify"
    avg_ms = prof["total_ms"] / max(1, prof["launches"])
    ach = prof["alg_bytes"] / max(1e-12, prof["total_ms"] / 1e3) / 1e9
    traffic, src, pl = None, "no engine index", None
    if key is not None and engine is not None:
        doc, src = find_profile(key)
        pl = profile_launches(doc, engine, merge_kernel, last=steps * tpp) if doc else None
        if doc is not None and pl is None:
            src = f"{src} holds fewer than {steps * tpp} launches of {merge_kernel} in engine {engine}"
        traffic = pl["hbm"] if pl else None
    return {"bound": "hbm", "kernel": merge_kernel + (" (SYNC launch, classification fused)"
                                                      if merge_kernel == "k_sync_apply" else ""),
            "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS, "traffic": traffic,
            **hbm_fields(traffic, avg_ms / 1e3),
            "traffic_unit": "HBM bytes per launch (mean over the timed periods' launches, per-launch PMC)",
            "traffic_source": src, "profiled_launch_us": pl["us"] if pl else None,
            "launches": prof["launches"], "avg_launch_ms": avg_ms,
            "alg_bytes_per_launch": prof["alg_bytes"] / max(1, prof["launches"]),
            # one SYNC merge launch per tick (the SYNC_ACK launch, k_ack_apply, reuses its results)
            "kernel_time_share": avg_ms * tpp / (dt * 1e3 / steps)}


def window_traffic(key, engine, kernels, launches):
    """the mean HBM bytes (and kernel-trace us) per round of the last `launches` launches of each of
    `kernels` (summed per round) in the profiled command's engine #engine"""
    doc, src = find_profile(key)
    if doc is None or engine is None:
        return None, src if doc is None else "no engine index", None
    tot = {"hbm": 0.0, "fetch": 0.0, "write": 0.0, "us": 0.0}
    for k in kernels:
        pl = profile_launches(doc, engine, k, last=launches)
        if pl is None:
            return None, f"{src} holds fewer than {launches} launches of {k} in engine {engine}", None
        for f in tot:
            tot[f] = None if tot[f] is None or pl[f] is None else tot[f] + pl[f]
    return tot, src, launches


def fanout_roofline(fprof, window, key=None, engine=None, launches=None):
    f_ms = fprof["total_ms"] / max(1, fprof["launches"])
    f_ach = fprof["alg_bytes"] / max(1e-12, fprof["total_ms"] / 1e3) / 1e9
    # traffic: the window's own launches in the per-launch PMC profile of this command and build
    w, src, _ = window_traffic(key, engine, ("k_gossip_emit",), launches)
    traffic = w["hbm"] if w else None
    msgs = fprof["messages"] / max(1, fprof["launches"])
    return {"bound": "hbm", "kernel": "k_gossip_emit", "achieved": f_ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": f_ach / HBM_PEAK_GBPS, "traffic": traffic, **hbm_fields(traffic, f_ms / 1e3),
            "traffic_source": src, "profiled_launch_us": w["us"] if w else None,
            "fetch_bytes_per_launch": w["fetch"] if w else None, "write_bytes_per_launch": w["write"] if w else None,
            "launches": fprof["launches"], "avg_launch_ms": f_ms,
            "alg_bytes_per_launch": fprof["alg_bytes"] / max(1, fprof["launches"]),
            "messages_per_launch": msgs,
            "states_per_launch": fprof["records"] / max(1, fprof["launches"]),
            "alg_bytes_rule": "24 B per materialised GOSSIP_REQ + 32 B per (gossip, sender round) state read",
            # the bytes the kernel must read and write: 16 hot bytes of every state it looks at (the
            # swept prefix and the in-window suffix, not all live states), 8 cold bytes and the 32-B
            # message of every materialised GOSSIP_REQ
            "must_read": must_read_fanout(fprof),
            "window": window}


def must_read_fanout(fprof):
    if not fprof.get("examined"):
        return None
    b = 16.0 * fprof["examined"] + 40.0 * fprof["messages"]
    ach = b / max(1e-12, fprof["total_ms"] / 1e3) / 1e9
    return {"bytes_per_launch": b / max(1, fprof["launches"]), "achieved": ach, "frac": ach / HBM_PEAK_GBPS,
            "examined_states_per_launch": fprof["examined"] / max(1, fprof["launches"]),
            "rule": "16 B per examined state (swept prefix + in-window suffix) + 8 B cold + 32 B message per "
                    "materialised GOSSIP_REQ"}


def deliver_roofline(dprof, window, key=None, engine=None, launches=None):
    """The delivery phase — k_deliver_coop (the biggest inboxes, a wave each) then k_gossip_deliver
    (every other inbox), timed together — over the same window as the fanout roofline:
    SURVEY.md §8(d) merge bytes, 24 B per delivered GOSSIP_REQ + 24 B (dedupe + view RMW) per message
    that runs the collector check (swim_profile_deliver)."""
    d_ms = dprof["total_ms"] / max(1, dprof["launches"])
    d_ach = dprof["alg_bytes"] / max(1e-12, dprof["total_ms"] / 1e3) / 1e9
    w, src, _ = window_traffic(key, engine, ("k_deliver_coop", "k_gossip_deliver"), launches)
    traffic = w["hbm"] if w else None
    msgs = dprof["messages"] / max(1, dprof["launches"])
    acc = dprof["records"] / max(1, dprof["launches"])
    return {"bound": "hbm", "kernel": "k_deliver_coop + k_gossip_deliver (one delivery phase)", "achieved": d_ach,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": d_ach / HBM_PEAK_GBPS, "traffic": traffic, **hbm_fields(traffic, d_ms / 1e3),
            "traffic_source": src, "profiled_launch_us": w["us"] if w else None,
            "traffic_over_alg": traffic / (dprof["alg_bytes"] / max(1, dprof["launches"])) if traffic else None,
            "fetch_bytes_per_message": w["fetch"] / msgs if w and w["fetch"] is not None and msgs else None,
            "write_bytes_per_accepted": w["write"] / acc if w and w["write"] is not None and acc else None,
            "launches": dprof["launches"], "avg_launch_ms": d_ms,
            "alg_bytes_per_launch": dprof["alg_bytes"] / max(1, dprof["launches"]),
            "messages_per_launch": msgs,
            "accepted_per_launch": acc,
            "alg_bytes_rule": "24 B per delivered GOSSIP_REQ + 24 B (8 B dedupe RMW + 16 B view RMW) per message "
                              "not flagged as a provable duplicate",
            "window": window}


def step_roofline(stats, prof, fprof, dprof, qprof, ticks, gossip_ticks, dt, steps, workload, n):
    """The whole step against the HBM roofline (the quiet step is a chain of latency-bound launches,
    no single kernel owns it): SURVEY.md §8(d)'s algorithmic bytes of everything the step did in the
    timed window — ping phase 21 B per ping, events 16 B each, timers 4 B per fired timer, and the
    sampled SYNC classify / fanout / delivery launches' per-launch bytes (swim_profile_*) times the
    window's launches of each — over the timed wall time.  `traffic`: the HBM bytes per tick of every
    kernel (the committed rocprofv3 PMC passes of this workload) times the window's ticks."""
    per = lambda p: p["alg_bytes"] / max(1, p["launches"])
    # the ticks that ran on the per-tick chain (the others ran inside quiet windows, whose bytes are
    # swim_profile_quiet's; the per-tick kernels are sampled one launch in three)
    chain = max(0, ticks - qprof["messages"])
    # pings of the ticks on the per-tick chain: the quiet windows' pings are inside their own bytes
    # (one ping per member-period they advanced, swim_profile_quiet's `records`)
    chain_pings = max(0, stats["pings"] - qprof["records"])
    parts = {"fd_pings": 21.0 * chain_pings, "events": 16.0 * stats["events"],
             "timers": 4.0 * stats["timers_fired"], "sync_classify": per(prof) * chain,
             "fanout": per(fprof) * gossip_ticks * chain / max(1, ticks), "deliver": per(dprof) * gossip_ticks * chain / max(1, ticks),
             "quiet_windows": float(qprof["alg_bytes"])}
    total = sum(parts.values())
    ach = total / dt / 1e9
    # (no HBM traffic here: the step is many launches of many kernels; the per-kernel rooflines carry
    # the profiled bytes of their own launches)
    traffic, src = None, "per kernel: see roofline, roofline_merge, roofline_fanout, roofline_deliver"
    return {"bound": "hbm", "scope": "step (one protocol period, every kernel)", "achieved": ach,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS,
            "traffic": traffic, "traffic_unit": "HBM bytes per step (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, all kernels)",
            "traffic_source": src, "alg_bytes_per_step": total / steps,
            "alg_bytes_per_member_period": total / steps / n,
            "alg_bytes_parts_per_step": {k: v / steps for k, v in parts.items()},
            "rule": "SURVEY.md §8(d): ping 21 B, event 16 B, timer 4 B, SYNC classify / fanout / delivery per "
                    "their swim_profile_* rules, quiet windows per swim_profile_quiet"}


def cpu_baseline(n, p0, periods, workload=None, single=True):
    """The CPU oracle (oracle/liboracle_swim.so, the C++ lockstep restatement) on the same N and
    workload, over the same periods the GPU timed ([p0, p0 + periods) of the schedule; the periods
    before p0 run untimed on all cores), bounded to `periods` periods: once with 1 thread and once
    multi-threaded over members (std::thread workers over member ranges in every phase; identical
    results, tests/test_golden.py).  The all-core figure is `value`."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    from swimgpu import abi
    lib = oracle.lib()
    workload = workload or WORKLOAD
    # the box's CPU share: OMP_NUM_THREADS is set to it there (os.cpu_count() is the whole machine)
    all_cores = max(1, min(64, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)))
    legs = {}
    for threads in ((1, all_cores) if single else (all_cores,)):
        cfg = make_config(lib)
        sch = Schedule(workload, n, p0 + periods)
        if workload == "churn":
            churn_capacities(cfg, sch.capacity)
        e = abi.Engine(lib, cfg, sch.capacity, n, 1)
        sch.setup(e)
        oracle.set_threads(e, all_cores)
        sch.run(e, 0, p0)
        oracle.set_threads(e, threads)
        t0 = time.perf_counter()
        sch.run(e, p0, p0 + periods)
        legs[threads] = time.perf_counter() - t0
        e.close()
    dt1, dtn = legs.get(1), legs[all_cores]
    out = {"value": n * periods / dtn, "unit": "member-periods/s", "cores": all_cores, "kind": "port",
           "nproc": os.cpu_count(), "cpu_model": cpu_model(),
           "sample": f"CPU oracle (C++ lockstep restatement), N={n}, LAN defaults, workload {workload}, "
                     f"periods {p0}..{p0 + periods} of the schedule (the GPU's first timed periods; "
                     f"0..{p0} untimed): {dtn:.1f} s on {all_cores} threads"
                     + (f", {dt1:.1f} s on 1 thread" if dt1 else "")}
    if dt1:
        out["single_thread_value"] = n * periods / dt1
    return out


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start `torch.distributed.run` with N ranks (one
    process per GPU) as a CHILD process — nothing here has touched the GPU yet — and return its exit
    code.  Rank 0's JSON line reaches stdout directly (the child inherits it)."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL and the exchange regions)
    return subprocess.run(cmd, env=env).returncode


def load_engine_hook(spec: str):
    """--engine-factory FILE.py:FN (test hook, CPU only): FN() returns a library exporting swim.h whose
    engines every rank runs UNSHARDED (the whole cluster on each rank), so the multi-process host
    path of this script — rank launch, rendezvous, barriers, max-over-ranks timing, the JSON line — is
    exercised without a GPU (tests/test_bench_launch.py)."""
    import importlib.util
    path, fn = spec.rsplit(":", 1)
    sp = importlib.util.spec_from_file_location("bench_engine_hook", path)
    mod = importlib.util.module_from_spec(sp)
    sp.loader.exec_module(mod)
    return getattr(mod, fn)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--members", type=int, default=None, help="default: 65,536 (16,384 for churn)")
    ap.add_argument("--cpu-periods", type=int, default=0, help="default: 10 (1 for churn)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="quiet workload: skip the fanout-roofline (failures window) and KS-mode side runs")
    ap.add_argument("--fanout-steps", type=int, default=6)
    ap.add_argument("--churn-steps", type=int, default=3, help="timed periods of the config-3 churn side run")
    ap.add_argument("--no-churn", action="store_true", help="skip the config-3 churn side run")
    ap.add_argument("--progress", action="store_true", help="print a stderr line after every period")
    ap.add_argument("--workload", choices=("quiet", "failures", "churn"), default="quiet")
    ap.add_argument("--gossip-capacity", type=int, default=0)
    ap.add_argument("--churn", type=int, default=None,
                    help="churn workload: members killed and joined per period (default 1%% of N, BASELINE config 3)")
    ap.add_argument("--loss", type=int, default=None, help="churn workload: uniform outbound loss %% (default 5)")
    ap.add_argument("--local-shards", type=int, default=1,
                    help="single-process sharded test rig (cfg.local_shards); measurement of the exchange only")
    ap.add_argument("--engine-factory", default=None, help=argparse.SUPPRESS)  # test hook, see load_engine_hook
    args = ap.parse_args()
    global WORKLOAD
    WORKLOAD = args.workload

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but this launch has WORLD_SIZE={world}")
    hook = load_engine_hook(args.engine_factory) if args.engine_factory else None

    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    if hook is None:
        torch.cuda.set_device(local_rank)

    import swimgpu
    from swimgpu import abi
    lib = hook() if hook else swimgpu.load_library()
    n = args.members or DEFAULT_MEMBERS[args.workload]
    sch = Schedule(args.workload, n, args.warmup + args.steps, args.churn, args.loss)
    sch.progress = args.progress
    cfg = make_config(lib, local_rank)
    cfg.gossip_capacity = args.gossip_capacity
    if args.workload == "churn":
        churn_capacities(cfg, sch.capacity)
        cfg.gossip_capacity = max(cfg.gossip_capacity, args.gossip_capacity)
    cfg.local_shards = args.local_shards
    se = None
    if world > 1:
        from swimgpu.dist import ShardedEngine
        factory = (lambda: abi.Engine(lib, cfg, sch.capacity, n, 1)) if hook else None
        se = ShardedEngine(lib, cfg, sch.capacity, n, 1, engine_factory=factory)
        e = se.engine
    else:
        e = abi.Engine(lib, cfg, sch.capacity, n, 1)
    shard = e.shard_info()
    if hook is None and shard["world"] != world * args.local_shards:
        raise SystemExit(f"bench.py: {world} ranks x {args.local_shards} local shards "
                         f"but the engine has {shard['world']} shards")
    sch.setup(e)

    def barrier():
        if world > 1:
            dist.barrier()
        if hook is None:
            torch.cuda.synchronize()

    def all_stats():
        return se.stats() if se is not None else e.stats()

    try:
        sch.run(e, 0, args.warmup)
        e.drain_events()
        barrier()
        e.profile_enable(True)
        st0 = all_stats()  # the timed window's counters are deltas from here (warmup excluded)
        qs0 = e.quiet_stats()
        barrier()
        t0 = time.perf_counter()
        sch.run(e, args.warmup, args.warmup + args.steps)
        barrier()
        dt = time.perf_counter() - t0
    except abi.SwimError as ex:
        raise SystemExit(f"{ex}; engine error bits {e.stats()['capacity_errors']:#x}")
    prof, fprof, dprof = e.profile_merge(), e.profile_fanout(), e.profile_deliver()
    st1 = all_stats()
    stats = {k: (st1[k] - st0[k] if k != "capacity_errors" else st1[k]) for k in st1}
    tpp = e.now()[2]
    e.drain_events()
    def reduce(p):  # summed over ranks (the line's kernel figures are the whole job's)
        st = torch.tensor([float(p["alg_bytes"]), p["total_ms"], float(p["launches"])], dtype=torch.float64)
        dist.all_reduce(st, op=dist.ReduceOp.SUM)
        return {**p, "alg_bytes": st[0].item(), "total_ms": st[1].item(), "launches": int(st[2].item())}
    if se is not None:
        dt = se.max_time(dt)
        prof, fprof, dprof = reduce(prof), reduce(fprof), reduce(dprof)
    if stats["capacity_errors"]:
        raise SystemExit(f"capacity error during the benchmark: {stats['capacity_errors']:#x}")

    qprof = e.profile_quiet()
    if se is not None:
        qprof = {**qprof, **reduce(qprof)}
    qst = e.quiet_stats()
    # the timed region's windows all precomputed by the one before: no k_quiet_scan ran in it
    timed_scans = (qst["windows"] - qs0["windows"]) - (qst.get("precomputed", 0) - qs0.get("precomputed", 0))
    value = n * args.steps / dt  # one cluster of n members, sharded over `world` GPUs
    ticks = args.steps * tpp
    gper = max(1, cfg.gossip_interval // e.now()[1])  # ticks per gossip round
    gossip_ticks = ticks // gper  # ticks with a gossip round
    line = {
        "metric": "simulated member-protocol-periods/sec at N=65,536; achieved HBM GB/s",
        "value": value,
        "unit": "member-periods/s",
        "n_gpus": world,
        "ranks": {"processes": world, "rccl_shards": shard["world"] if hook is None else None,
                  "launch": "torch.distributed.run, one process per GPU" if world > 1 else "single process"},
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": WORKLOAD_TEXT[args.workload].format(n=n, churn=sch.churn, every=KILL_EVERY,
                                                                   loss=sch.loss),
                   "members": n, "tick_ms": 100,
                   "parallelism": (f"rows sharded over {world} GPUs, RCCL send/recv over xGMI" if world > 1 else
                                   f"single GPU, {args.local_shards} in-process shards" if args.local_shards > 1
                                   else "single GPU")},
        "timing": "every kernel time on this line is HIP events on the engine's own stream, measured in this "
                  "run; profiles/<round>_*_kernel_stats.csv (rocprofv3 --kernel-trace --stats of the same command) "
                  "must agree with them; PMC passes give traffic only (their durations include counter overhead)",
        "roofline": None,
        "quiet_windows": {"ticks": qst["ticks"], "windows": qst["windows"], "attempts": qst["attempts"],
                          "cut_short": qst["cut_short"], "precomputed": qst.get("precomputed", 0),
                          "timed_ticks": ticks},
        "stats": {k: stats[k] for k in ("syncs", "sync_records", "gossip_messages", "gossips_created", "pings",
                                         "timers_fired", "events")},
    }
    step = step_roofline(stats, prof, fprof, dprof, qprof, ticks, gossip_ticks, dt, args.steps, args.workload, n)
    # the roofline of the step's dominant kernels: the quiet windows' (k_quiet_scan + k_quiet_apply)
    # when they carried the step, else the whole per-tick chain against its wall time
    # the timed window's launches in the profiled command: after the warm-up's — k_quiet_apply once per
    # window ATTEMPT (an attempt that advances no tick launches it too) and per local shard,
    # k_quiet_scan once per attempt whose end was not precomputed, per local shard
    key = bench_key(args, n)
    first = timed_launch_index(qs0, args.local_shards)
    line["bench_key"] = key
    line["build"] = build_hash()
    line["roofline"] = quiet_roofline(qprof, key, scanned=timed_scans > 0, first=first) \
        if qprof["launches"] else step
    line["roofline_step"] = step
    # per-tick kernel launches of the timed window, in the main engine (engine #0 of the profile)
    gticks = gossip_ticks if args.workload != "quiet" or not qprof["launches"] else 0
    if prof["launches"]:
        line["roofline_merge"] = merge_roofline(prof, world, args.local_shards, dt, args.steps, tpp, key,
                                                0 if args.local_shards == 1 and world == 1 else None)
    if fprof["alg_bytes"] > 0:
        # the gossip fanout kernel (north_star: merge AND fanout against the HBM roofline); only
        # workloads with gossip traffic (failures, churn) give it work
        eng = 0 if args.local_shards == 1 and world == 1 and args.workload == "failures" else None
        line["roofline_fanout"] = fanout_roofline(fprof, f"the timed window ({args.workload})", key, eng, gticks)
        line["roofline_deliver"] = deliver_roofline(dprof, f"the timed window ({args.workload})", key, eng, gticks)
    if args.workload == "quiet" and qprof["launches"] and hook is None:
        line["steady_state"] = steady_state(e, sch, args, n, dt, barrier, se)
    if world == 1 and args.workload == "quiet" and qprof["launches"] and hook is None:
        line["quiet_window_model"] = quiet_window_model(e, n, tpp)
    if world == 1 and args.workload == "quiet" and not args.no_extras and args.local_shards == 1 and hook is None:
        e.close()
        # (1) the per-tick kernel chain on the same workload and the same timed periods (quiet windows
        # off): the SYNC merge's roofline (k_sync_apply's SYNC launch, classification fused) is
        # measured there
        # (the engines of this command in creation order: #0 the headline's, #1 this one, #2 failures,
        # #3 churn, then KS mode; a profile's per-launch lists are kept per engine)
        p_dt, p_prof, _, _, _, _ = side_run(lib, "quiet", n, args.warmup, args.steps, local_rank, quiet=False)
        line["per_tick_path"] = {
            "value": n * args.steps / p_dt, "unit": "member-periods/s", "ms_per_step": p_dt / args.steps * 1e3,
            "steps": args.steps, "warmup": args.warmup,
            "config": "same workload and timed periods, quiet windows off (swim_set_quiet_path(0)): the per-tick "
                      "kernel chain of DESIGN.md §5",
            "roofline_merge": merge_roofline(p_prof, 1, 1, p_dt, args.steps, tpp, key, 1)}
        # (2) the failures workload over a window that starts with its second kill (period 30: FD
        # detection, the SUSPECT storm through all N members, the gossip's remaining rounds): the
        # fanout and delivery kernels.  The first storm also holds every member's first
        # selectGossipMembers shuffle of its 65,535-entry remote list, which is not the steady state.
        fw, fs = KILL_FIRST + KILL_EVERY, args.fanout_steps
        f_dt, _, f_fprof, f_st, f_dprof, _ = side_run(lib, "failures", n, fw, fs, local_rank)
        window = (f"config4-lan-failures N={n}: periods {fw}..{fw + fs} (member killed at period {fw}), "
                  f"{f_st['gossip_messages']} GOSSIP_REQs sent")
        line["failures"] = {"value": n * fs / f_dt, "unit": "member-periods/s", "ms_per_step": f_dt / fs * 1e3,
                            "steps": fs, "window": window,
                            "roofline_fanout": fanout_roofline(f_fprof, window, key, 2, fs * tpp // gper),
                            "roofline_deliver": deliver_roofline(f_dprof, window, key, 2, fs * tpp // gper)}
        line["roofline_fanout"] = line["failures"]["roofline_fanout"]
        line["roofline_deliver"] = line["failures"]["roofline_deliver"]
        # (3) BASELINE config 3 (churn) at its stated N = 16,384: periods 1..1 + churn_steps (the SYNC
        # re-gossip storm grows every period)
        if not args.no_churn:
            cs = args.churn_steps
            c_pt = []
            c_dt, _, _, c_st, _, _ = side_run(lib, "churn", DEFAULT_MEMBERS["churn"], 1, cs, local_rank,
                                              period_times=c_pt)
            line["churn"] = {"value": DEFAULT_MEMBERS["churn"] * cs / c_dt, "unit": "member-periods/s",
                             "ms_per_step": c_dt * 1e3 / cs, "steps": cs, "warmup": 1,
                             # each timed period (1, 2, ...): the storm grows every period, so the CPU
                             # baseline below (period 1 on the oracle) compares with period 1 only
                             "ms_per_period": [round(t * 1e3, 3) for t in c_pt],
                             "config": WORKLOAD_TEXT["churn"].format(n=DEFAULT_MEMBERS["churn"],
                                                                     churn=DEFAULT_MEMBERS["churn"] * CHURN_PER_MILLE // 1000,
                                                                     loss=CHURN_LOSS),
                             "gossip_messages": c_st["gossip_messages"]}
        # (4) the timing mode whose latency distributions pass the KS test against the reference-timing
        # DES (tests/test_ks_des.py: independent timer phases, 10 ms ticks); same quiet workload
        k_dt, _, _, _, _, k_q = side_run(lib, "quiet", n, args.warmup, args.steps, local_rank, timer_stagger=1,
                                         tick_ms=10)
        line["ks_mode"] = {"value": n * args.steps / k_dt, "unit": "member-periods/s",
                           "ms_per_step": k_dt / args.steps * 1e3, "steps": args.steps, "warmup": args.warmup,
                           "quiet_windows": k_q,
                           "config": "same workload, timer_stagger=1, tick_ms=10 (100 ticks per period)",
                           "ks": "tests/test_ks_des.py::test_ks_gpu_vs_des (N=64 and 1,024, 200 seeds, p >= 0.01)"}
    if hook is not None:
        line["engine"] = f"TEST HOOK {args.engine_factory}: not a measurement"
    if rank == 0 and world == 1 and not args.no_cpu_baseline and hook is None:
        e.close()
        # churn: the oracle needs minutes per period once the storm builds, so the sample is the
        # first timed period only
        cpu_periods = args.cpu_periods or (1 if args.workload == "churn" else 10)
        line["cpu_baseline"] = cpu_baseline(n, args.warmup, min(cpu_periods, args.steps))
        if "churn" in line:  # config 3's first timed period on the oracle, all cores (the GPU side run's period 1)
            line["churn"]["cpu_baseline"] = cpu_baseline(DEFAULT_MEMBERS["churn"], 1, 1, "churn", single=False)
            if line["churn"].get("ms_per_period"):  # the same period on the GPU
                line["churn"]["cpu_baseline"]["gpu_same_period_value"] = (
                    DEFAULT_MEMBERS["churn"] / (line["churn"]["ms_per_period"][0] / 1e3))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
