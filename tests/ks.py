"""Detection-latency and convergence distributions: lockstep engine vs reference-timing DES.

BASELINE.json's north_star asks detection-latency and convergence distributions to match "within a
stated KS tolerance wherever reference scheduling is nondeterministic"; SURVEY.md §8 fixes the
statistics and the bar: two-sample Kolmogorov-Smirnov, pass at p >= 0.01.  The reference cannot run
here (no JVM), so its timing is restated by oracle/des.py (asynchronous, random timer phases,
message delays, timeout races); the lockstep side is any engine behind include/swim.h (the C++
oracle on CPU, libswimgpu.so on the GPU).

Per run one member is killed and four statistics are taken (ms after the kill), from one randomly
chosen live viewer so that every sample is independent:
  detect    first FailureDetector SUSPECT of the victim (any member),
  suspect   the viewer's table first shows the victim SUSPECT (FD or gossip),
  removed   the viewer emits REMOVED for the victim,
  converge  the last live member emits REMOVED (all live views agree).
Lockstep times are tick * tick_ms; the kill lands uniformly inside a tick of the real cluster, so
lockstep latencies are measured from the middle of the kill tick.
"""
from __future__ import annotations

import random

import numpy as np
from scipy import stats as sps

import des
from swimgpu import abi

STATS = ("detect", "suspect", "removed", "converge")
P_MIN = 0.01  # pass at p >= 0.01


def _draw(n, seed, tpp):
    rng = random.Random(seed * 7919 + 17)
    victim = rng.randrange(n)
    viewer = rng.choice([x for x in range(n) if x != victim])
    return victim, viewer, rng.randrange(tpp)


def lockstep_sample(lib, n, seed, horizon_ms, **cfg_overrides):
    """One lockstep run on `lib` (oracle or libswimgpu.so) with the same draw rule as the DES."""
    cfg = abi.default_config(lib, 0, record_fd_events=1, **cfg_overrides)
    with abi.Engine(lib, cfg, n, n, seed) as e:
        _, tick_ms, tpp = e.now()
        victim, viewer, phase = _draw(n, seed, tpp)
        e.step_ticks(100 + phase)  # 10 s of converged running, kill inside a random tick of the period
        e.drain_events()
        t_kill, _, _ = e.now()
        e.kill(victim)
        horizon = int(horizon_ms // tick_ms)
        t_sus = None
        for _ in range(horizon):  # the viewer's table is polled tick by tick until it shows SUSPECT
            e.step_ticks(1)
            st = int(abi.cell_status(e.read_view(viewer)[victim]))
            if st == 1:
                t_sus = e.now()[0]
                break
        rest = t_kill + horizon - e.now()[0]
        if rest > 0:
            e.step_ticks(rest)
        ev = e.drain_events()
    at = lambda t: (int(t) - int(t_kill)) * tick_ms - tick_ms / 2  # noqa: E731
    fd = ev[(ev["type"] == abi.EV_FD_SUSPECT) & (ev["subject"] == victim)]
    rem = ev[(ev["type"] == abi.EV_REMOVED) & (ev["subject"] == victim)]
    rem_v = rem[rem["viewer"] == viewer]
    return {"detect": at(fd["tick"].min()) if len(fd) else None,
            "suspect": at(t_sus) if t_sus is not None else None,
            "removed": at(rem_v["tick"].min()) if len(rem_v) else None,
            "converge": at(rem["tick"].max()) if len(np.unique(rem["viewer"])) == n - 1 else None}


def des_sample(n, seed, horizon_ms):
    return des.des_sample(n, seed, horizon_ms)


def collect(sampler, seeds):
    out = {k: [] for k in STATS}
    for s in seeds:
        r = sampler(s)
        for k in STATS:
            out[k].append(r[k])
    return out


def compare(a, b):
    """KS per statistic; a run that never reached a statistic fails it (both sides must finish)."""
    res = {}
    for k in STATS:
        xa, xb = a[k], b[k]
        missing = sum(x is None for x in xa) + sum(x is None for x in xb)
        xa = np.array([x for x in xa if x is not None], dtype=float)
        xb = np.array([x for x in xb if x is not None], dtype=float)
        r = sps.ks_2samp(xa, xb)
        res[k] = {"D": float(r.statistic), "p": float(r.pvalue), "missing": missing,
                  "median_lockstep": float(np.median(xa)), "median_des": float(np.median(xb))}
    return res
