"""The reference's own scenario tests, restated on the lockstep oracle and on the GPU engine (virtual time).

Each test mirrors one JUnit test: same topology, same fault schedule, same test configuration, and
the same final-state assertions (trusted / suspected sets, event sequences, FD event statuses).
Wall-clock sleeps (BaseTest.awaitSeconds / awaitSuspicion) become virtual-time steps.  The same
scenarios run bit-exactly on the GPU in test_gpu_parity.py / test_gpu_scenarios.py.
"""
import pytest

import oracle
from swimgpu import abi
from swimgpu.cluster import ClusterConfig, ClusterMath, MembershipEvent, MemberStatus, SimulatedCluster

Type = MembershipEvent.Type


# Every restatement runs on the CPU oracle and, marked gpu, on libswimgpu.so itself: the reference's
# own assertions are then checked on the MI355X engine directly, not only through oracle parity.
@pytest.fixture(autouse=True, params=["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def backend(request, monkeypatch):
    if request.param == "gpu":
        from swimgpu import load_library
        glib = load_library()
        monkeypatch.setattr(oracle, "lib", lambda: glib)
    return request.param

# MembershipProtocolTest.testConfig (:1111-1121)
PING_INTERVAL = 200
TEST_SYNC_INTERVAL = 500


def mp_config(n):
    return (ClusterConfig.default_config()
            .membership(seed_members=tuple(range(n)), sync_interval=TEST_SYNC_INTERVAL, sync_timeout=100)
            .failure_detector(ping_interval=PING_INTERVAL, ping_timeout=100)
            .with_metadata_timeout(100))


# FailureDetectorTest.createFd (:401-408): local config, pingTimeout 100, pingInterval 200, 2 relays.
# The FD tests run the detector against a static member list; a huge suspicion multiplier keeps the
# full stack from removing suspected members during the test window.
def fd_config():
    return (ClusterConfig.default_local_config()
            .failure_detector(ping_timeout=100, ping_interval=200, ping_req_members=2)
            .membership(suspicion_mult=1000))


def make(config, n, seed=1, engine=None, lib=None, **knobs):
    lib = lib or oracle.lib()
    cfg = config.to_abi(lib, record_fd_events=1, **knobs)
    e = engine or abi.Engine(lib, cfg, n, n, seed)
    return SimulatedCluster.from_engine(e, config)


def trusted(c, m):
    return sorted(x.id for x in c.membership(m).members_by_status(MemberStatus.ALIVE))


def suspected(c, m):
    return sorted(x.id for x in c.membership(m).members_by_status(MemberStatus.SUSPECT))


def next_fd_status(c, m, others):
    """FailureDetectorTest.listenNextEventFor: first FD event per other member."""
    first = {}
    for ev in c.failure_detector(m).listen():
        first.setdefault(ev.member.id, ev.status)
    return {o: first.get(o) for o in others}


# ------------------------------------------------------------------------------ FailureDetectorTest
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fd_trusted(seed):  # :51-78
    c = make(fd_config(), 3, seed)
    c.step(4)
    for m in range(3):
        assert set(next_fd_status(c, m, [o for o in range(3) if o != m]).values()) == {MemberStatus.ALIVE}


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fd_suspected(seed):  # :80-115
    c = make(fd_config(), 3, seed)
    for m in range(3):
        c.network_emulator(m).block_outbound(0, 1, 2)
    c.step(2)
    for m in range(3):
        assert set(next_fd_status(c, m, [o for o in range(3) if o != m]).values()) == {MemberStatus.SUSPECT}


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_fd_trusted_despite_bad_network(seed):  # :117-147
    c = make(fd_config(), 3, seed)
    c.network_emulator(0).block_outbound(1)
    c.step(4)
    for m in range(3):
        evs = c.failure_detector(m).listen()
        assert evs and all(e.status == MemberStatus.ALIVE for e in evs)


def test_fd_suspected_member_with_bad_network_gets_partitioned():  # :180-240
    c = make(fd_config(), 4, 7)
    c.network_emulator(0).block_outbound(0, 1, 2, 3)
    c.step(4)
    assert set(next_fd_status(c, 0, [1, 2, 3]).values()) == {MemberStatus.SUSPECT}
    for m in (1, 2, 3):
        assert next_fd_status(c, m, [0])[0] == MemberStatus.SUSPECT
    c.network_emulator(0).unblock_all_outbound()
    c.await_seconds(4)
    c.step(0)
    for m in range(4):
        c.failure_detector(m).listen()
    c.step(4)
    for m in range(4):
        assert set(next_fd_status(c, m, [o for o in range(4) if o != m]).values()) == {MemberStatus.ALIVE}


def test_fd_suspected_member_with_normal_network_gets_partitioned():  # :242-300
    c = make(fd_config(), 4, 8)
    for m in (0, 1, 2):
        c.network_emulator(m).block_outbound(3)
    c.step(4)
    for m in (0, 1, 2):
        assert next_fd_status(c, m, [3])[3] == MemberStatus.SUSPECT
    assert set(next_fd_status(c, 3, [0, 1, 2]).values()) == {MemberStatus.SUSPECT}
    for m in (0, 1, 2):
        c.network_emulator(m).unblock_all_outbound()
    c.await_seconds(4)
    for m in range(4):
        c.failure_detector(m).listen()
    c.step(4)
    for m in range(4):
        assert set(next_fd_status(c, m, [o for o in range(4) if o != m]).values()) == {MemberStatus.ALIVE}


def test_fd_member_status_change_after_network_recovery():  # :302-342
    c = make(fd_config(), 2, 9)
    c.network_emulator(0).block_outbound(1)
    c.network_emulator(1).block_outbound(0)
    c.step(2)
    assert next_fd_status(c, 0, [1])[1] == MemberStatus.SUSPECT
    assert next_fd_status(c, 1, [0])[0] == MemberStatus.SUSPECT
    c.network_emulator(0).unblock_all_outbound()
    c.network_emulator(1).unblock_all_outbound()
    c.await_seconds(2)
    c.failure_detector(0).listen()
    c.failure_detector(1).listen()
    c.step(2)
    assert next_fd_status(c, 0, [1])[1] == MemberStatus.ALIVE
    assert next_fd_status(c, 1, [0])[0] == MemberStatus.ALIVE


# ------------------------------------------------------------------------------ MembershipProtocolTest
def test_mp_initial_phase_ok():  # :259-282
    c = make(mp_config(3), 3)
    c.await_seconds(1)
    for m in range(3):
        assert trusted(c, m) == [0, 1, 2] and suspected(c, m) == []


def test_mp_network_partition_due_no_outbound_then_recover():  # :284-328
    c = make(mp_config(3), 3, 2)
    c.await_seconds(3)
    for m in range(3):
        c.network_emulator(m).block_outbound(0, 1, 2)
    c.await_suspicion(3)
    for m in range(3):
        assert trusted(c, m) == [m] and suspected(c, m) == []
    for m in range(3):
        c.network_emulator(m).unblock_all_outbound()
    c.await_seconds(TEST_SYNC_INTERVAL * 2 / 1000)
    for m in range(3):
        assert trusted(c, m) == [0, 1, 2] and suspected(c, m) == []


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mp_member_lost_network_due_no_outbound_then_recover(seed):  # :330-384
    c = make(mp_config(3), 3, seed)
    c.await_seconds(1)
    for m in range(3):
        assert trusted(c, m) == [0, 1, 2]
    c.network_emulator(1).block_outbound(0, 2)
    c.network_emulator(0).block_outbound(1)
    c.network_emulator(2).block_outbound(1)
    c.await_seconds(1)
    assert trusted(c, 0) == [0, 2] and suspected(c, 0) == [1]
    assert trusted(c, 1) == [1] and suspected(c, 1) == [0, 2]
    assert trusted(c, 2) == [0, 2] and suspected(c, 2) == [1]
    for m in range(3):
        c.network_emulator(m).unblock_all_outbound()
    c.await_seconds(1)
    for m in range(3):
        assert trusted(c, m) == [0, 1, 2] and suspected(c, m) == []


def test_mp_network_partition_twice_due_no_outbound_then_recover():  # :386-454
    c = make(mp_config(3), 3, 4)
    c.await_seconds(1)
    c.network_emulator(1).block_outbound(0, 2)
    c.network_emulator(0).block_outbound(1)
    c.network_emulator(2).block_outbound(1)
    c.await_seconds(1)
    assert suspected(c, 0) == [1] and suspected(c, 1) == [0, 2] and suspected(c, 2) == [1]
    c.network_emulator(0).block_outbound(2)
    c.network_emulator(2).block_outbound(0)
    c.await_seconds(1)
    for m in range(3):
        assert trusted(c, m) == [m] and suspected(c, m) == [o for o in range(3) if o != m]
    for m in range(3):
        c.network_emulator(m).unblock_all_outbound()
    c.await_seconds(1)
    for m in range(3):
        assert trusted(c, m) == [0, 1, 2] and suspected(c, m) == []


def test_mp_long_network_partition_due_no_outbound_then_removed():  # :511-562
    c = make(mp_config(4), 4, 5)
    c.await_seconds(1)
    c.network_emulator(0).block_outbound(2, 3)
    c.network_emulator(1).block_outbound(2, 3)
    c.network_emulator(2).block_outbound(0, 1)
    c.network_emulator(3).block_outbound(0, 1)
    c.await_seconds(2)
    assert trusted(c, 0) == [0, 1] and suspected(c, 0) == [2, 3]
    assert trusted(c, 2) == [2, 3] and suspected(c, 2) == [0, 1]
    c.await_suspicion(4)
    for m, side in ((0, [0, 1]), (1, [0, 1]), (2, [2, 3]), (3, [2, 3])):
        assert trusted(c, m) == side and suspected(c, m) == []


def test_mp_network_partition_many_due_no_inbound_then_removed_then_recover():  # :1035-1109
    c = make(mp_config(4), 4, 6)
    c.await_seconds(1)
    for m in range(4):
        c.membership(m).listen()
    for m in range(4):
        c.network_emulator(m).block_all_inbound()
    c.await_seconds(2)
    for m in range(4):
        assert trusted(c, m) == [m] and suspected(c, m) == [o for o in range(4) if o != m]
    c.await_suspicion(4)
    for m in range(4):
        removed = sorted(e.member.id for e in c.membership(m).listen() if e.is_removed())
        assert removed == [o for o in range(4) if o != m]
    for m in range(4):
        c.network_emulator(m).unblock_all_inbound()
    c.await_seconds(3)
    for m in range(4):
        assert trusted(c, m) == [0, 1, 2, 3] and suspected(c, m) == []


def test_mp_leave_cluster():  # :73-105
    c = make(mp_config(3), 3, 7)
    c.await_seconds(2)
    for m in range(3):
        c.membership(m).listen()
    c.shutdown(1)
    c.await_seconds(2)
    c.await_suspicion(3)
    for m in (0, 2):
        evs = [e for e in c.membership(m).listen() if not e.is_added()]
        assert [(e.member.id, e.type) for e in evs[:2]] == [(1, Type.LEAVING), (1, Type.REMOVED)]


# ------------------------------------------------------------------------------ BASELINE configs
def test_config1_three_members_kill_one():
    """BASELINE config 1: LAN defaults, kill member 1 at period 5; both survivors remove it."""
    c = make(ClusterConfig.default_lan_config(), 3, 11)
    c.step(5)
    c.kill(1)
    c.step(25)
    for m in (0, 2):
        evs = c.membership(m).listen()
        assert [(e.member.id, e.type) for e in evs] == [(1, Type.REMOVED)]
        assert trusted(c, m) == [0, 2]
        # removal lands after suspicion timeout (5 * ceilLog2(3) * 1 s = 10 s) + detection
        assert 15_000 <= evs[0].timestamp <= 18_000


def test_config2_1024_single_failure_converges():
    """BASELINE config 2: 1,024 members, kill 17 at period 10; every live member removes it once,
    within detection + suspicion timeout (55 s at N=1024) + gossip dissemination."""
    lib = oracle.lib()
    c = make(ClusterConfig.default_lan_config(), 1024, 2, lib=lib)
    c.step(10)
    c.kill(17)
    c.step(140)
    removed = {v: [e for e in c.membership(v).listen() if e.is_removed()] for v in range(1024)}
    assert all(len(removed[v]) == 1 and removed[v][0].member.id == 17 for v in range(1024) if v != 17)
    t_rem = [removed[v][0].timestamp / 1000 for v in range(1024) if v != 17]
    assert min(t_rem) >= 10 + 55 and max(t_rem) <= 10 + 55 + 20


# ------------------------------------------------------------------------------ GossipProtocolTest
# testGossipProtocol (:107-199) over the experiment rows (:47-63) whose mean delay (2 ms) is below
# one 100 ms tick; the default outbound loss on every member; one gossip from member 0.
@pytest.mark.parametrize("n,loss", [(2, 0), (3, 0), (5, 0), (10, 0), (10, 10), (10, 25), (10, 50), (50, 0),
                                    (50, 10)])
def test_gossip_protocol_experiment(n, loss):
    c = make(ClusterConfig.default_config(), n, seed=3)
    for m in range(n):
        c.network_emulator(m).set_default_outbound_settings(loss, 0)
    gcfg = c.config.gossip_config
    timeout_ms = ClusterMath.gossip_timeout_to_sweep(gcfg.gossip_repeat_mult, n, gcfg.gossip_interval)
    data = "test gossip - 7"
    fut = c.gossip(0).spread(data)
    t0 = c.now_ms
    receivers, dissemination = {}, None

    def pump():
        nonlocal dissemination
        for m in range(n):
            for g in c.gossip(m).listen():
                if g.data == data:
                    receivers[m] = receivers.get(m, 0) + 1
        if dissemination is None and len(receivers) == n - 1:
            dissemination = c.now_ms - t0

    while c.now_ms - t0 < 2 * timeout_ms and dissemination is None:  # latch.await(2 * gossipTimeout)
        c.step_ticks(1)
        pump()
    assert len(receivers) == n - 1 and 0 not in receivers, "Not all members received gossip"
    assert dissemination < timeout_ms, f"Too long dissemination time {dissemination}ms (timeout {timeout_ms}ms)"
    # awaitFullCompletion: the gossip's whole lifetime plus three gossip intervals
    c.await_seconds((timeout_ms - dissemination + 3 * gcfg.gossip_interval) / 1000)
    pump()
    assert all(k == 1 for k in receivers.values()), "Delivered gossip twice to same member"
    assert fut.done  # spread()'s Mono completed at the originator


def gossip_only_config():
    """GossipProtocolTest / GossipDelayTest run GossipProtocolImpl alone over a static member list
    (initGossipProtocol :274-295): the failure detector and SYNC are pushed past the test window."""
    return (ClusterConfig.default_config()
            .failure_detector(ping_interval=3_600_000, ping_timeout=500)
            .membership(sync_interval=3_600_000))


# GossipProtocolTest rows with a 100 ms mean delay (:47-63): delays quantised to the 100 ms tick
@pytest.mark.parametrize("n,loss,delay", [(10, 25, 100), (50, 10, 100), (10, 0, 300)])
def test_gossip_protocol_experiment_delayed(n, loss, delay):
    c = make(gossip_only_config(), n, seed=5)
    for m in range(n):
        c.network_emulator(m).set_default_outbound_settings(loss, delay)
    gcfg = c.config.gossip_config
    timeout_ms = ClusterMath.gossip_timeout_to_sweep(gcfg.gossip_repeat_mult, n, gcfg.gossip_interval)
    data = "delayed gossip"
    fut = c.gossip(0).spread(data)
    t0 = c.now_ms
    receivers, dissemination = {}, None
    while c.now_ms - t0 < 2 * timeout_ms:
        c.step_ticks(1)
        for m in range(n):
            for g in c.gossip(m).listen():
                if g.data == data:
                    receivers[m] = receivers.get(m, 0) + 1
        if dissemination is None and len(receivers) == n - 1:
            dissemination = c.now_ms - t0
    assert len(receivers) == n - 1 and 0 not in receivers, "Not all members received gossip"
    assert dissemination < timeout_ms
    assert all(k == 1 for k in receivers.values()), "Delivered gossip twice to same member"
    assert fut.done


# GossipDelayTest.testMessageDelayMoreThanGossipSweepTime (:33-69): members 0 and 1 delay every
# outbound message by 3,000 ms on average, member 2 by 100 ms; member 0 spreads three gossips
def test_gossip_delay_more_than_sweep_time():
    c = make(gossip_only_config(), 3, seed=9)
    for m, d in ((0, 3000), (1, 3000), (2, 100)):
        c.network_emulator(m).set_default_outbound_settings(0, d)
    for i in range(3):
        c.gossip(0).spread(f"message: {i}")
    gcfg = c.config.gossip_config
    sweep_ms = ClusterMath.gossip_timeout_to_sweep(gcfg.gossip_repeat_mult, 3, gcfg.gossip_interval)
    counts = [0, 0, 0]
    ticks = 2 * (sweep_ms + 6000) // c.tick_ms
    for _ in range(ticks):
        c.step_ticks(1)
        for m in range(3):
            counts[m] += len(c.gossip(m).listen())
    assert counts == [0, 3, 3]


# FailureDetectorTest-style: a slow link (mean delay well above the ping timeout) makes the direct
# ping time out, yet the member stays trusted through the relays; a fast one answers directly
def test_fd_delay_trusted_through_relays():
    c = make(fd_config(), 4, seed=11)
    c.network_emulator(0).outbound_settings(1, 0, 2000)  # 0 -> 1 slow
    c.await_seconds(10)
    fd = c.failure_detector(0).listen()
    statuses = {ev.status for ev in fd if ev.member.id == 1}
    assert MemberStatus.ALIVE in statuses
    assert trusted(c, 0) == [0, 1, 2, 3]


# ------------------------------------------------------------------------------ ClusterNamespacesTest
@pytest.mark.parametrize("ns", ["", "  ", "/abc", "a /b /c", "a\nb\nc", ".abc", "abc.", "a-/b-/c-", "a+/b+/c+",
                                "abc/", "abc/*", "abc/.", "./abc", "a./b./c."])
def test_invalid_namespace_format(ns):  # testInvalidNamespaceFormat (:20-56)
    from swimgpu.cluster import validate_namespace
    with pytest.raises(ValueError, match="membership.namespace format is invalid"):
        validate_namespace(ns)


def _namespace_cluster(namespaces, seeds):
    """Members start one by one (startAwait) through the seeds; member 0 is up from the start."""
    n = len(namespaces)
    lib = oracle.lib()
    cfg = mp_config(n).to_abi(lib)
    e = abi.Engine(lib, cfg, n, 1, 1)
    e.set_seeds(list(seeds))
    c = SimulatedCluster.from_engine(e, mp_config(n).membership(seed_members=tuple(seeds)))
    c.set_namespaces(namespaces)
    for m in range(1, n):
        c.join(m)
        c.step_ticks(3)
    c.await_seconds(2)
    return c


def others(c, m):
    return sorted(x.id for x in c.membership(m).other_members())


def test_separate_empty_namespaces():  # :58-81
    c = _namespace_cluster(["root", "root1", "root2"], seeds=(0,))
    assert others(c, 0) == others(c, 1) == others(c, 2) == []


def test_separate_non_empty_namespaces():  # :84-143
    c = _namespace_cluster(["root", "root", "root", "root2", "root2", "root2"], seeds=(0, 1, 2, 3, 4))
    assert (others(c, 0), others(c, 1), others(c, 2)) == ([1, 2], [0, 2], [0, 1])
    assert (others(c, 3), others(c, 4), others(c, 5)) == ([4, 5], [3, 5], [3, 4])


def test_simple_namespaces_hierarchy():  # :146-196
    c = _namespace_cluster(["develop", "develop/develop", "develop/develop", "develop/develop-2",
                            "develop/develop-2"], seeds=(0, 1, 2, 3))
    assert others(c, 0) == [1, 2, 3, 4]
    assert (others(c, 1), others(c, 2)) == ([0, 2], [0, 1])
    assert (others(c, 3), others(c, 4)) == ([0, 4], [0, 3])


def test_isolated_parent_namespaces():  # :199-250
    c = _namespace_cluster(["a/1", "a/1/c", "a/1/c", "a/111", "a/111/c", "a/111/c"], seeds=(0, 1, 2, 3, 4))
    assert (others(c, 0), others(c, 1), others(c, 2)) == ([1, 2], [0, 2], [0, 1])
    assert (others(c, 3), others(c, 4), others(c, 5)) == ([4, 5], [3, 5], [3, 4])


# ---- per-member seed lists (MembershipProtocolTest.createMembership(transport, testConfig(seeds)),
# :1123-1177: every member its own ClusterConfig; start().block() — members start one after another)
def _start_seeded(n, seeds_of, before_start=None):
    lib = oracle.lib()
    base = mp_config(n).membership(seed_members=())
    e = abi.Engine(lib, base.to_abi(lib, record_fd_events=1), n, 1, 1)
    c = SimulatedCluster.from_engine(e, base)
    c.set_member_config(0, mp_config(n).membership(seed_members=tuple(seeds_of[0])))
    if before_start:
        before_start(c)
    for m in range(1, n):
        c.join(m, config=mp_config(n).membership(seed_members=tuple(seeds_of[m])))
        c.step_ticks(3)  # start().block(): the initial SYNCs answered or timed out (syncTimeout 100 ms)
    return c


def test_mp_limited_seed_members():  # testLimitedSeedMembers (:713-743)
    # A: no seeds; B, C: seed A; D, E: seed B
    c = _start_seeded(5, [[], [0], [0], [1], [1]])
    c.await_seconds(3)
    for m in range(5):
        assert trusted(c, m) == [0, 1, 2, 3, 4] and suspected(c, m) == []


def test_mp_node_join_cluster_with_no_inbound():  # testNodeJoinClusterWithNoInbound (:788-813)
    # C blocks all inbound before it starts: A admits nobody whose metadata it cannot fetch (its
    # SYNC_ACK to C waits for that fetch, then C drops it), so C stays alone and A / B never add it
    c = _start_seeded(3, [[], [0], [0]], before_start=lambda c: c.network_emulator(2).block_all_inbound())
    c.await_seconds(3)
    assert trusted(c, 0) == [0, 1] and trusted(c, 1) == [0, 1]
    assert trusted(c, 2) == [2] and suspected(c, 2) == []


# ------------------------------------------------------------------------------ ClusterTest
def test_update_metadata():  # testUpdateMetadata (:179-247): every member sees the new metadata
    n = 12
    lib = oracle.lib()
    e = abi.Engine(lib, ClusterConfig.default_config().to_abi(lib), n, 2, 1)
    e.set_seeds([0])
    c = SimulatedCluster.from_engine(e, ClusterConfig.default_config().membership(seed_members=(0,)))
    for m in range(2, n):
        c.join(m)
    c.await_seconds(3)
    for m in range(n):
        c.membership(m).listen()
    c.update_metadata(1)
    c.await_seconds(3)
    for m in range(n):
        ev = c.membership(m).listen()
        upd = [x for x in ev if x.type == Type.UPDATED]
        assert ([x.member.id for x in upd] == [1]) == (m != 1), (m, ev)
        assert not [x for x in ev if x.type != Type.UPDATED]
    assert c.membership(1).incarnation() == 1  # updateIncarnation: ALIVE inc 0 -> 1


def test_mp_restart_stopped_members():  # MembershipProtocolTest.testRestartStoppedMembers (:564-640)
    """C and D stop, are suspected, then REMOVED after the suspicion timeout; restarted instances
    (new ids at new addresses: free slots 4 and 5, seeded with the original four addresses) join and
    every live member trusts exactly {A, B, new C, new D}."""
    lib = oracle.lib()
    conf = mp_config(4)
    e = abi.Engine(lib, conf.to_abi(lib, record_fd_events=1), 6, 4, 9)
    c = SimulatedCluster.from_engine(e, conf)
    c.await_seconds(1)
    assert trusted(c, 0) == [0, 1, 2, 3]
    c.membership(0).listen(), c.membership(1).listen()
    c.kill(2)
    c.kill(3)
    c.await_seconds(1)
    assert trusted(c, 0) == [0, 1] and suspected(c, 0) == [2, 3]
    assert trusted(c, 1) == [0, 1] and suspected(c, 1) == [2, 3]
    c.await_suspicion(4)
    for m in (0, 1):
        assert trusted(c, m) == [0, 1] and suspected(c, m) == []
        removed = sorted(x.member.id for x in c.membership(m).listen() if x.type == Type.REMOVED)
        assert removed == [2, 3]
    c.join(4)
    c.join(5)
    c.await_seconds(3)
    for m, want in ((4, [0, 1, 4, 5]), (5, [0, 1, 4, 5]), (0, [0, 1, 4, 5]), (1, [0, 1, 4, 5])):
        assert trusted(c, m) == want and suspected(c, m) == [], m


def restart_on_same_addresses(lib, seed=9):
    """MembershipProtocolTest.testRestartStoppedMembersOnSameAddresses (:643-711): C and D stop and
    are suspected; new instances (fresh ids: free slots 4 and 5) start on C's and D's ports."""
    conf = mp_config(4)
    e = abi.Engine(lib, conf.to_abi(lib, record_fd_events=1), 6, 4, seed)
    c = SimulatedCluster.from_engine(e, conf)
    c.await_seconds(1)
    for m, want in ((0, [0, 1, 2, 3]), (1, [0, 1, 2, 3]), (2, [0, 1, 2, 3]), (3, [0, 1, 2, 3])):
        assert trusted(c, m) == want, m
    c.membership(0).listen(), c.membership(1).listen()
    c.failure_detector(0).listen(), c.failure_detector(1).listen()
    c.kill(2)
    c.kill(3)
    c.await_seconds(1)
    for m in (0, 1):
        assert trusted(c, m) == [0, 1] and suspected(c, m) == [2, 3], m
    c.join(4, same_address_as=2)
    c.join(5, same_address_as=3)
    return c


def test_mp_restart_stopped_members_on_same_addresses():
    c = restart_on_same_addresses(oracle.lib())
    t_restart = c.now_ms
    c.await_seconds(3)
    # new C -> A, B, new D; new D -> A, B, new C; A, B -> B / A, new C, new D; nobody suspected
    for m, want in ((4, [0, 1, 4, 5]), (5, [0, 1, 4, 5]), (0, [0, 1, 4, 5]), (1, [0, 1, 4, 5])):
        assert trusted(c, m) == want and suspected(c, m) == [], m
    for m in (0, 1):
        ev = c.membership(m).listen()
        assert sorted(x.member.id for x in ev if x.type == Type.REMOVED) == [2, 3]
        # old C / D are removed through DEST_GONE: a ping to their address reaches the new member,
        # which answers DEST_GONE (FailureDetectorImpl.onPing :227-259) -> FD DEAD (:382-404) ->
        # REMOVED well before their suspicion timeouts (ClusterMath.suspicionTimeout: 3 s here)
        fd = c.failure_detector(m).listen()
        dead = {x.member.id for x in fd if x.status == MemberStatus.DEAD}
        assert dead == {2, 3}, (m, fd)
        removed_ms = [x.timestamp for x in ev if x.type == Type.REMOVED]
        assert max(removed_ms) - t_restart < 1500, removed_ms
    # the restarted members never admit the old records at their own addresses (:605-610)
    assert 2 not in [x.id for x in c.membership(4).members()]
    assert 3 not in [x.id for x in c.membership(5).members()]
