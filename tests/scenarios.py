"""Deterministic lockstep scenarios shared by the oracle tests, the GPU parity tests and the
golden-fixture generator.  Each restates a configuration of BASELINE.json or a scenario of the
reference's own test suites (FailureDetectorTest, MembershipProtocolTest, GossipProtocolTest) as a
schedule of control operations at given ticks.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from swimgpu import abi


@dataclasses.dataclass
class Scenario:
    name: str
    capacity: int
    n_initial: int
    ticks: int
    seed: int = 1
    preset: int = 0
    cfg: dict = dataclasses.field(default_factory=dict)
    seeds: tuple = ()
    ops: list = dataclasses.field(default_factory=list)  # (tick, op, args...) applied before tick+1
    check_every: int = 10
    shardable: bool = True  # False: uses a feature sharded engines do not have


def apply_op(e: abi.Engine, op, args):
    if op == "kill":
        e.kill(*args)
    elif op == "leave":
        e.leave(*args)
    elif op == "join":
        e.join(*args)
    elif op == "join_at":
        e.join_at(*args)
    elif op == "loss":
        e.set_default_loss(*args)
    elif op == "link_loss":
        e.set_link_loss(*args)
    elif op == "link_in":
        e.set_link_inbound(*args)
    elif op == "default_in":
        e.set_default_inbound(*args)
    elif op == "update_meta":
        e.update_metadata(*args)
    elif op == "namespaces":
        from swimgpu.cluster import namespaces_related
        names = sorted(set(args[0]))
        gid = {x: i for i, x in enumerate(names)}
        rel = np.array([[namespaces_related(x, y) for y in names] for x in names], dtype=np.uint8)
        e.set_namespaces(np.array([gid[x] for x in args[0]], dtype=np.uint16), rel)
    elif op == "member_seeds":  # (m, [seeds] or None): member m's own seedMembers
        e.set_member_seeds(args[0], None if args[1] is None else list(args[1]))
    elif op == "default_delay":
        e.set_default_delay(*args)
    elif op == "link_delay":
        e.set_link_delay(*args)
    elif op == "spread":
        e.spread(*args)
    elif op == "partition":
        e.set_partition(None if args[0] is None else np.asarray(args[0], dtype=np.uint16))
    elif op == "ingest":  # (viewer, [(member, status, inc), ...], initial): an external SYNC_ACK off the wire
        from swimgpu import wire
        v, recs, initial = args
        d = wire.Directory.local(e.capacity)
        stranger = wire.MembershipRecord(wire.Member("f" * 8, "elsewhere:4800"), abi.ALIVE, 0)  # not a slot: dropped
        data = wire.SyncData(tuple(wire.MembershipRecord(d.member(m), st, inc) for m, st, inc in recs) + (stranger,))
        msg = wire.Message(((wire.HEADER_QUALIFIER, wire.SYNC_ACK), (wire.HEADER_SENDER, "elsewhere:4800")), data)
        e.ingest_sync(v, wire.engine_records(wire.deserialize(wire.serialize(msg)), d), initial)
    else:
        raise ValueError(op)


def make_engine(lib, sc: Scenario, rccl: bool = False) -> abi.Engine:
    """rccl: an RCCL engine of one rank (swim_create_shard with a comm id at world 1; GPU library)"""
    cfg = abi.default_config(lib, sc.preset, **sc.cfg)
    if rccl:
        e = abi.Engine(lib, cfg, sc.capacity, sc.n_initial, sc.seed, rank=0, world=1,
                       comm_id=abi.comm_unique_id(lib))
    else:
        e = abi.Engine(lib, cfg, sc.capacity, sc.n_initial, sc.seed)
    if sc.seeds:
        e.set_seeds(list(sc.seeds))
    return e


def run(e: abi.Engine, sc: Scenario, on_check=None):
    """Advance `e` through the scenario; call on_check(tick) every check_every ticks and at the end."""
    ops = sorted(sc.ops, key=lambda x: x[0])
    t = 0
    oi = 0
    while t < sc.ticks:
        while oi < len(ops) and ops[oi][0] <= t:
            apply_op(e, ops[oi][1], ops[oi][2:])
            oi += 1
        nxt = min(sc.ticks, t + sc.check_every)
        if oi < len(ops):
            nxt = min(nxt, max(ops[oi][0], t + 1))
        e.step_ticks(nxt - t)
        t = nxt
        if on_check and (t % sc.check_every == 0 or t == sc.ticks):
            on_check(t)


def _partition(n, split):
    g = np.zeros(n, dtype=np.uint16)
    g[split:] = 1
    return g


ALL_ = abi.ALL_MEMBERS


def catalog() -> list[Scenario]:
    """Small scenarios (oracle-fast) used for bit-exact parity."""
    fd_test = dict(ping_interval=200, ping_timeout=100, ping_req_members=2, gossip_interval=100,
                   gossip_repeat_mult=2, sync_interval=15000, suspicion_mult=3, metadata_timeout=1000,
                   record_fd_events=1)
    mp_test = dict(sync_interval=500, sync_timeout=100, ping_interval=200, ping_timeout=100, metadata_timeout=100,
                   record_fd_events=1)
    return [
        # BASELINE config 1: 3 members, LAN defaults, kill member 1 at period 5, run 30 periods
        Scenario("config1_kill", 3, 3, 300, seed=11, ops=[(50, "kill", 1)]),
        # FailureDetectorTest.testTrustedDespiteBadNetwork (:117-147): A->B outbound blocked
        Scenario("fd_trusted_despite_bad_network", 3, 3, 60, seed=3, cfg=fd_test, ops=[(0, "link_loss", 0, 1, 100)]),
        # FailureDetectorTest.testSuspected (:80-115): all outbound blocked
        Scenario("fd_all_blocked", 3, 3, 80, seed=4, cfg=fd_test,
                 ops=[(0, "link_loss", a, b, 100) for a in range(3) for b in range(3)]),
        # FailureDetectorTest.testSuspectedMemberWithBadNetworkGetsPartitioned (:180-240) + recovery
        Scenario("fd_isolated_then_recover", 4, 4, 160, seed=5, cfg=fd_test,
                 ops=[(0, "link_loss", 0, b, 100) for b in range(4)] + [(40, "link_loss", 0, b, -1) for b in range(4)]),
        # MembershipProtocolTest.testMemberLostNetworkDueNoOutboundThenRecover (:330-384)
        Scenario("mp_member_lost_network", 3, 3, 40, seed=6, cfg=mp_test, seeds=(0, 1, 2),
                 ops=[(10, "link_loss", 1, 0, 100), (10, "link_loss", 1, 2, 100), (10, "link_loss", 0, 1, 100),
                      (10, "link_loss", 2, 1, 100), (20, "link_loss", 1, 0, -1), (20, "link_loss", 1, 2, -1),
                      (20, "link_loss", 0, 1, -1), (20, "link_loss", 2, 1, -1)]),
        # MembershipProtocolTest.testLongNetworkPartitionDueNoOutboundThenRemoved (:511-562)
        Scenario("mp_long_partition_removed", 4, 4, 700, seed=7, cfg=mp_test, seeds=(0, 1, 2, 3),
                 ops=[(20, "partition", [0, 0, 1, 1]), (600, "partition", None)]),
        # MembershipProtocolTest.testNetworkPartitionManyDueNoInboundThenRemovedThenRecover (:1035-1109)
        Scenario("mp_inbound_blocked_removed_recover", 4, 4, 700, seed=8, cfg=mp_test, seeds=(0, 1, 2, 3),
                 ops=[(20, "default_in", 0, abi.ALL_MEMBERS), (400, "default_in", 1, abi.ALL_MEMBERS)]),
        # MembershipProtocolTest.testLeaveCluster (:73-105): graceful shutdown -> LEAVING, REMOVED
        Scenario("mp_leave_cluster", 3, 3, 400, seed=9, cfg=mp_test, seeds=(0, 1, 2), ops=[(40, "leave", 1, 1)]),
        # joins through seeds (MembershipProtocolTest.testInitialPhaseOk :259-282, limited seeds)
        Scenario("mp_joins_via_seed", 12, 6, 400, seed=10, cfg=mp_test, seeds=(0,),
                 ops=[(5, "join", 6), (5, "join", 7), (23, "join", 8), (41, "join", 9), (41, "join", 10),
                      (77, "join", 11), (150, "kill", 3)]),
        # 64 members, 5 % uniform loss + kills, LAN defaults (config 3 in miniature)
        Scenario("loss5_kills_64", 64, 64, 600, seed=12, cfg=dict(record_fd_events=1),
                 ops=[(0, "loss", 5, abi.ALL_MEMBERS), (100, "kill", 9), (250, "kill", 40), (300, "kill", 41)],
                 check_every=50),
        # 48 members, churn: kills and joins through two seeds under 2 % loss
        Scenario("churn_48", 48, 40, 800, seed=13, seeds=(0, 1),
                 ops=[(0, "loss", 2, abi.ALL_MEMBERS)] + [(60 * i, "kill", 2 + 3 * i) for i in range(1, 6)]
                 + [(60 * i + 7, "join", 39 + i) for i in range(1, 9)] + [(333, "leave", 20, 1)],
                 check_every=50),
        # join burst through one seed under loss: the seed's ALIVE gossips reach members out of order,
        # so collectors spill into interval blocks (tier growth, merge back inline, block recycling)
        Scenario("join_burst_144", 144, 64, 260, seed=22, seeds=(0,),
                 ops=[(0, "loss", 10, abi.ALL_MEMBERS)] + [(5, "join", 64 + i) for i in range(80)],
                 check_every=20),
        # the same with gossipSegmentationThreshold = 8: collectors cleared by checkGossipSegmentation, and
        # gossips re-accepted afterwards (GossipState.infected grows past its first sender)
        Scenario("join_burst_seg", 144, 64, 260, seed=23, seeds=(0,),
                 cfg=dict(gossip_segmentation_threshold=8, gossip_capacity=4096),
                 ops=[(0, "loss", 10, abi.ALL_MEMBERS)] + [(5, "join", 64 + i) for i in range(80)],
                 check_every=20),
        # BASELINE config 3's rates in miniature: 5 % uniform outbound loss, every period 1 % of the
        # members (2 of 200) killed and as many fresh members joined through seed 0, for 25 periods,
        # then 35 quiet periods (the kills' suspicion timers fire, REMOVED)
        Scenario("config3_rates_200", 250, 200, 600, seed=15, seeds=(0,),
                 cfg=dict(gossip_capacity=8192, timer_capacity=1 << 16),
                 ops=[(0, "loss", 5, abi.ALL_MEMBERS)]
                 + [(10 * p, "kill", (7 + 13 * p + 100 * j) % 200) for p in range(1, 26) for j in range(2)]
                 + [(10 * p, "join", 200 + 2 * (p - 1) + j) for p in range(1, 26) for j in range(2)],
                 check_every=50),
        # user gossips (GossipProtocol.spread / listen) under 25 % loss: GossipProtocolTest's N=10 row
        # (:47-63), three gossips from three members, one while another is still spreading
        Scenario("user_gossip_10_loss25", 10, 10, 160, seed=16,
                 ops=[(0, "loss", 25, abi.ALL_MEMBERS), (5, "spread", 0, 101), (5, "spread", 3, 102),
                      (12, "spread", 7, 103)], check_every=20),
        # GossipDelayTest (:33-69): members 0 and 1 delay every message by 3 s on average, member 2 by
        # 100 ms; member 0 spreads three gossips (failure detector and SYNC pushed past the window)
        Scenario("gossip_delay_3", 3, 3, 190, seed=17, cfg=dict(ping_interval=3_600_000, sync_interval=3_600_000),
                 ops=[(0, "default_delay", 3000, 0), (0, "default_delay", 3000, 1), (0, "default_delay", 100, 2),
                      (1, "spread", 0, 1), (1, "spread", 0, 2), (1, "spread", 0, 3)],
                 check_every=20),
        # the whole stack under delay: a 150 ms mean delay on every message (round trips beyond the
        # 500 ms ping timeout, late direct acks racing the relays, gossips arriving on non-gossip
        # ticks), a slow link, 5 % loss, a kill, a user gossip
        Scenario("delay_fd_gossip_12", 12, 12, 700, seed=18,
                 ops=[(0, "default_delay", 150, abi.ALL_MEMBERS), (0, "loss", 5, abi.ALL_MEMBERS),
                      (0, "link_delay", 2, 5, 2500), (50, "spread", 4, 77), (120, "kill", 9)],
                 check_every=50),
        # ClusterTest.testUpdateMetadata (:179-247): members join through seed 0, member 1 updates its
        # metadata twice (updateIncarnation: ALIVE inc+1 gossiped; every viewer fetches -> UPDATED)
        Scenario("update_metadata_12", 12, 2, 300, seed=19, seeds=(0,), cfg=mp_test,
                 ops=[(2, "join", 2 + i) for i in range(10)] + [(60, "update_meta", 1), (140, "update_meta", 1),
                                                               (141, "kill", 7)],
                 check_every=20),
        # ClusterNamespacesTest.testSimpleNamespacesHierarchy (:149-196) + testSeparateNonEmptyNamespaces
        # (:84-143) on one engine: "develop" sees everyone below it, siblings stay apart, "root" and
        # "root2" never meet; members start one by one through seeds
        Scenario("namespaces_9", 9, 1, 240, seed=20, seeds=(0, 1, 2, 5, 6, 7), cfg=mp_test,
                 ops=[(0, "namespaces", ["develop", "develop/develop", "develop/develop", "develop/develop-2",
                                         "develop/develop-2", "root", "root", "root2", "root2"])]
                 + [(2 + 3 * i, "join", 1 + i) for i in range(8)],
                 check_every=20),
        # MembershipProtocolTest.testRestartStoppedMembersOnSameAddresses (:643-711): C and D stop, new
        # instances start on their ports; pings to the old ids answer DEST_GONE -> DEAD -> REMOVED
        Scenario("mp_restart_same_address", 6, 4, 60, seed=24, cfg=mp_test, seeds=(0, 1, 2, 3),
                 ops=[(10, "kill", 2), (10, "kill", 3), (20, "join_at", 4, 2), (20, "join_at", 5, 3)]),
        # restarts on the same address under 5 % loss (DEST_GONE through ping-req relays, unanswered
        # metadata requests): a seed restarted, a member restarted twice, a plain kill and join
        Scenario("restart_same_address_40", 40, 32, 600, seed=25, seeds=(0, 5),
                 ops=[(0, "loss", 5, abi.ALL_MEMBERS), (30, "kill", 5), (30, "kill", 9), (45, "join_at", 32, 5),
                      (60, "join_at", 33, 9), (100, "kill", 12), (110, "join", 35), (200, "kill", 33),
                      (215, "join_at", 34, 9)],
                 check_every=50),
        # the same under a 150 ms mean message delay (a DEST_GONE ack arriving late, after the ping
        # timeout, joins the ping-req race)
        Scenario("restart_same_address_delay", 40, 32, 600, seed=26, seeds=(0, 5), cfg=dict(delay_capacity=16384),
                 ops=[(0, "loss", 5, abi.ALL_MEMBERS), (0, "default_delay", 150, abi.ALL_MEMBERS), (30, "kill", 5),
                      (30, "kill", 9), (45, "join_at", 32, 5), (60, "join_at", 33, 9), (200, "kill", 33),
                      (215, "join_at", 34, 9)],
                 check_every=50),
        # SYNC / SYNC_ACK and GET_METADATA under delay (NetworkEmulatorTransport :59-75 delays every
        # send and requestResponse): a 120 ms mean on every link, a 600 ms link, 2 % loss; members join
        # through two seeds (initial SYNCs answered late or timed out), a kill, a metadata update (every
        # viewer's fetch races the 300 ms metadata timeout)
        Scenario("sync_delay_24", 24, 16, 420, seed=27, seeds=(0, 3),
                 cfg=dict(sync_interval=2000, sync_timeout=300, ping_interval=600, ping_timeout=300,
                          metadata_timeout=300, record_fd_events=1, delay_capacity=16384),
                 ops=[(0, "default_delay", 120, abi.ALL_MEMBERS), (0, "loss", 2, abi.ALL_MEMBERS),
                      (0, "link_delay", 3, 0, 600), (4, "join", 16), (9, "join", 17), (9, "join", 18),
                      (30, "join", 19), (31, "join", 20), (60, "kill", 7), (80, "update_meta", 2),
                      (150, "join", 21), (150, "join", 22), (151, "join", 23)],
                 check_every=20),
        # NetworkEmulatorTransport applies the receiver's inbound filter when a message ARRIVES
        # (listen :78-83, requestResponse :72-74), and the transport's send after tryDelayOutbound
        # meets a receiver that stopped meanwhile: inbound blocks switched on and off while delayed
        # GOSSIP_REQs, SYNCs / SYNC_ACKs (a joiner's initial SYNCs among them) and FD acks are in
        # flight, a seed stopped while the joiners' initial SYNCs travel to it
        Scenario("inbound_block_in_flight_16", 16, 12, 400, seed=28, seeds=(0, 2),
                 cfg=dict(sync_interval=1000, sync_timeout=600, ping_interval=600, ping_timeout=300,
                          metadata_timeout=2000, record_fd_events=1, delay_capacity=16384),
                 ops=[(0, "default_delay", 200, ALL_), (0, "link_delay", 4, 1, 900), (9, "spread", 2, 55),
                      (10, "default_in", 0, 3), (12, "join", 12), (12, "join", 13), (13, "default_in", 1, 3),
                      (14, "kill", 2), (30, "link_in", 5, 1, 0), (33, "link_in", 5, 1, -1),
                      (50, "spread", 6, 56), (51, "default_in", 0, 7), (53, "default_in", 1, 7),
                      (70, "link_in", 1, 4, 0), (74, "link_in", 1, 4, -1), (90, "join", 14),
                      (91, "default_in", 0, 0), (95, "default_in", 1, 0)],
                 check_every=20),
        # SYNC_ACKs from outside the simulation (swim_ingest_sync, onSyncAck MembershipProtocolImpl.java
        # :363-391) decoded from the wire: a SUSPECT record of a live member (suspicion timer), one of the
        # viewer itself (refutation, inc+1 gossip), a LEAVING record, ALIVE records of a stopped slot
        # (metadata fetch fails) and of a fresh joiner (fetch, ADDED), a stale record, an initial-sync
        # ingestion, SUSPECT of a just-killed member, an empty table, a higher incarnation under delay
        Scenario("external_sync_16", 16, 12, 320, seed=29, seeds=(0,), cfg=mp_test,
                 ops=[(15, "ingest", 3, [(5, abi.SUSPECT, 1), (3, abi.SUSPECT, 0), (7, abi.LEAVING, 1),
                                         (12, abi.ALIVE, 0), (9, abi.ALIVE, 0)], False),
                      (25, "join", 12), (26, "ingest", 9, [(12, abi.ALIVE, 0), (13, abi.ALIVE, 0)], True),
                      (60, "kill", 4), (61, "ingest", 1, [(4, abi.SUSPECT, 0)], False), (100, "ingest", 6, [], False),
                      (120, "default_delay", 80, ALL_), (121, "ingest", 2, [(11, abi.ALIVE, 5), (10, abi.SUSPECT, 0)],
                                                                     False),
                      (200, "ingest", 8, [(5, abi.LEAVING, 0), (14, abi.SUSPECT, 3)], False),
                      # two ingestions at one viewer between the same ticks: the second one's events and
                      # metadata-fetch draws continue the first one's (distinct keys, distinct draws)
                      (250, "ingest", 3, [(6, abi.LEAVING, 9), (10, abi.ALIVE, 9)], False),
                      (250, "ingest", 3, [(9, abi.LEAVING, 9), (11, abi.ALIVE, 12)], False)],
                 check_every=20),
        # onSync's SYNC_ACK waits for the SYNC's updateMembership Monos (MembershipProtocolImpl.java
        # :394-415, :491-509): admissions whose metadata fetch is lost (10 % loss: the request fails at
        # once, a lost response waits out metadataTimeout), refused (member 1 drops everything from seed
        # 0) or answered late; a LEAVING record learned by SYNC (member 7 was deaf while 5 left) waits
        # for the re-gossip to spread; joiners' start0 Flux (:250-291) waits for its initial merges'
        # fetches, or times out with fetches in flight (seed 3 slow: a 1.5 s link)
        Scenario("sync_ack_waits_24", 24, 16, 500, seed=30, seeds=(0, 3),
                 cfg=dict(sync_interval=1000, sync_timeout=1000, ping_interval=600, ping_timeout=300,
                          metadata_timeout=400, record_fd_events=1, delay_capacity=16384),
                 ops=[(0, "loss", 10, ALL_), (2, "link_in", 1, 0, 0), (5, "join", 16), (5, "join", 17),
                      (9, "join", 18), (20, "default_in", 0, 7), (30, "leave", 5, 1), (45, "default_in", 1, 7),
                      (60, "join", 19), (100, "kill", 11), (150, "join", 20), (150, "join", 21),
                      (200, "link_delay", 3, 22, 1500), (200, "link_delay", 22, 3, 1500), (201, "join", 22),
                      (230, "default_delay", 150, 8), (231, "join", 23), (300, "link_in", 1, 0, -1)],
                 check_every=20),
        # per-member seedMembers (each member's own ClusterConfig; MembershipProtocolTest
        # .testLimitedSeedMembers :713-743 in a bigger cluster): joiners seeded by different members,
        # one by a chain (17 -> 16 -> 8), one with its own address among its seeds (dropped,
        # cleanUpSeedMembers :171-190), one with a dead seed, one with no seeds (alone until someone
        # SYNCs to it), one put back on the engine-wide list; 5 % loss
        Scenario("member_seeds_20", 20, 6, 400, seed=31, seeds=(0,),
                 cfg=dict(sync_interval=1000, sync_timeout=500, ping_interval=600, ping_timeout=300,
                          metadata_timeout=500, record_fd_events=1),
                 ops=[(0, "loss", 5, ALL_), (0, "member_seeds", 3, [5, 4]), (2, "member_seeds", 6, [1]),
                      (2, "member_seeds", 7, [2, 1, 2]), (2, "member_seeds", 8, [6]), (3, "join", 6), (3, "join", 7),
                      (6, "join", 8), (10, "kill", 4), (11, "member_seeds", 9, [4, 5]), (11, "join", 9),
                      (20, "member_seeds", 10, [10, 3]), (20, "join", 10), (30, "member_seeds", 11, []),
                      (30, "join", 11), (40, "member_seeds", 12, [11]), (40, "join", 12),
                      (60, "member_seeds", 16, [8]), (60, "join", 16), (70, "member_seeds", 17, [16]),
                      (70, "join", 17), (90, "member_seeds", 13, [2]), (91, "member_seeds", 13, None),
                      (91, "join", 13), (120, "member_seeds", 1, [17]), (200, "join", 14)],
                 check_every=20),
        # a join burst under message delay: 160 members join through one seed at once, and each
        # joiner's first SYNC_ACK admits the whole table through delayed GET_METADATA round trips
        # (46 K round trips in 25 ticks, several thousand in flight together, beyond the delayed-fetch queue's base capacity of 4,096: the
        # engine grows it before the joins' tick, grow_for_joins) — and the seed holds the 160
        # joiners' SYNC_ACKs at once while their admission fetches run (pending acks beyond the base 64)
        Scenario("join_burst_delay_256", 256, 96, 30, seed=32, seeds=(0,),
                 cfg=dict(sync_interval=3000, sync_timeout=1000, ping_interval=1000, ping_timeout=500,
                          metadata_timeout=1000, delay_capacity=1 << 20, gossip_capacity=8192),
                 ops=[(0, "default_delay", 200, ALL_)] + [(5, "join", m) for m in range(96, 256)],
                 check_every=10),
        # 2-way partition held past the suspicion timeout, heal via SYNC through seeds (config 5 in miniature)
        Scenario("partition_heal_32", 32, 32, 1600, seed=14, seeds=(0, 16),
                 cfg=dict(sync_interval=5000), ops=[(100, "partition", _partition(32, 16)), (1100, "partition", None)],
                 check_every=100),
    ]


CONFIG2_MEMBERS = list(range(0, 1024, 37)) + [17, 18, 255, 256, 1023]  # rows compared at N = 1,024


def config2() -> Scenario:
    """BASELINE config 2: 1,024 members, 0 % loss, kill member 17 at period 10, 150 periods."""
    return Scenario("config2_1024", 1024, 1024, 1500, seed=2, ops=[(100, "kill", 17)], check_every=100)
