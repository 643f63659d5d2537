"""Message delay on the SYNC / SYNC_ACK and GET_METADATA legs (NetworkEmulatorTransport.send /
requestResponse :50-75 delay every message): the lockstep rules of DESIGN.md §3, on the CPU oracle
and (marked gpu) on libswimgpu.so.

* start0's initial sync (MembershipProtocolImpl.java:268-289): Flux.timeout(syncTimeout) restarts at
  every answer, so a joiner whose seeds answer late starts its periodic sync syncTimeout after the
  start (or after its last answer), and stays without periodic sync while it waits;
* MetadataStoreImpl.fetchMetadata (:146-185): a round trip that reaches metadataTimeout fails, so the
  ALIVE admission it guards is skipped.
"""
import pytest

import oracle
from swimgpu import abi


@pytest.fixture(params=["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def lib(request):
    if request.param == "gpu":
        from swimgpu import load_library
        return load_library()
    return oracle.lib()


# 100 ms ticks: sync 1 s, syncTimeout 300 ms (3 ticks), ping 200 / 100 ms
CFG = dict(sync_interval=1000, sync_timeout=300, ping_interval=200, ping_timeout=100, metadata_timeout=300)


def engine(lib, n, n_initial, seed, **kw):
    cfg = abi.default_config(lib, 0, **{**CFG, **kw})
    return abi.Engine(lib, cfg, n, n_initial, seed)


def test_initial_sync_waits_then_times_out(lib):
    """Seeds 0 and 1 answer through a 5 s mean delay: the joiner's answers arrive after syncTimeout
    (P(one answer within 300 ms) ~ 6 % per seed; seed 5 draws none), so its periodic sync is off while
    it waits and starts at the start tick + syncTimeout."""
    e = engine(lib, 3, 2, seed=5)
    e.set_seeds([0, 1])
    e.set_default_delay(5000, 0)
    e.set_default_delay(5000, 1)
    e.join(2)
    e.step_ticks(1)  # start0 at tick 1
    t0 = 1
    m = e.read_member(2)
    assert m["sync_on"] == 0  # the Flux is still subscribed
    e.step_ticks(1)
    assert e.read_member(2)["sync_on"] == 0
    e.step_ticks(2)
    m = e.read_member(2)
    assert m["sync_on"] == 1 and m["sync_start"] == t0 + 3


def test_initial_sync_without_delay_decides_at_start(lib):
    """No delay: every initial SYNC resolves within the start tick, the periodic sync starts then."""
    e = engine(lib, 3, 2, seed=5)
    e.set_seeds([0, 1])
    e.join(2)
    e.step_ticks(1)
    m = e.read_member(2)
    assert m["sync_on"] == 1 and m["sync_start"] == 1


def test_initial_sync_answered_late_starts_at_last_answer(lib):
    """A 150 ms mean on the seeds: every answer arrives within the timeout of the previous one for
    this seed, and the periodic sync starts at the tick of the last answer."""
    e = engine(lib, 3, 2, seed=11)
    e.set_seeds([0, 1])
    e.set_default_delay(150, 0)
    e.set_default_delay(150, 1)
    e.join(2)
    ticks = []
    for t in range(1, 12):
        e.step_ticks(1)
        m = e.read_member(2)
        ticks.append((t, m["sync_on"], m["sync_start"]))
    done = [t for t, on, _ in ticks if on]
    assert done, ticks
    start = ticks[done[0] - 1][2]
    assert 1 <= start <= done[0] and start < 1 + 3 * 2, ticks  # an answer, not a timeout chain


def test_metadata_fetch_fails_past_timeout(lib):
    """A 3 s mean on every link against a 300 ms metadata timeout: almost every fetch of the joiners'
    ALIVE admissions fails; without delay none does."""
    slow = engine(lib, 12, 4, seed=3)
    slow.set_seeds([0])
    slow.set_default_delay(3000, abi.ALL_MEMBERS)
    fast = engine(lib, 12, 4, seed=3)
    fast.set_seeds([0])
    for e in (slow, fast):
        for m in range(4, 12):
            e.join(m)
        e.step_ticks(120)
    s, f = slow.stats(), fast.stats()
    assert f["fetches"] > 0 and f["fetch_ok"] == f["fetches"]
    assert s["fetches"] > 0 and s["fetch_ok"] < 0.3 * s["fetches"]


def test_refused_delay_mean_changes_nothing(lib):
    """A mean above the engine's tick cap (SWIM_DELAY_MEAN_MAX_TICKS ticks, swim_delay.h) is refused
    with SWIM_EINVAL and leaves the engine exactly as it was: no delay machinery switched on, so a
    joiner's start0 Flux still decides at its start tick (MembershipProtocolImpl.java:268-289) and the
    run equals one where the call was never made."""
    def run(refuse):
        e = engine(lib, 3, 2, seed=5)
        e.set_seeds([0, 1])
        if refuse:
            for call in (lambda: e.set_default_delay(10 ** 6, 0), lambda: e.set_default_delay(10 ** 6),
                         lambda: e.set_link_delay(0, 1, 10 ** 6)):
                with pytest.raises(abi.SwimError) as ex:
                    call()
                assert ex.value.code == abi.SWIM_EINVAL
        e.join(2)
        e.step_ticks(40)
        return e, [e.read_member(m) for m in range(3)], e.stats(), e.drain_events()
    a, ma, sa, ea = run(False)
    b, mb, sb, eb = run(True)
    assert mb[2]["sync_on"] == 1 and mb[2]["sync_start"] == 1
    assert ma == mb and sa == sb
    assert ea.tobytes() == eb.tobytes()
