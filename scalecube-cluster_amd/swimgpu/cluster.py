"""Host-side mirror of scalecube-cluster's public protocol API over the engine ABI.

Names, argument meaning and error behaviour follow the reference:
  ClusterConfig / FailureDetectorConfig / GossipConfig / MembershipConfig
      (cluster-api/.../ClusterConfig.java:25-428, fdetector/FailureDetectorConfig.java,
       gossip/GossipConfig.java, membership/MembershipConfig.java) — immutable, clone-on-write
  ClusterMath (cluster/.../ClusterMath.java:8-136)
  Member (Member.java:16-143), MemberStatus (MemberStatus.java:3-19)
  MembershipEvent (membership/MembershipEvent.java:13-148)
  MembershipProtocol view: member(), members(), otherMembers(), member(id), listen()
      (membership/MembershipProtocol.java:14-65) + getMembershipRecords() (Impl :903-905)
  FailureDetector view: listen() of FailureDetectorEvents (fdetector/FailureDetector.java:12-25)
  NetworkEmulator (cluster-testlib/.../NetworkEmulator.java): outbound loss / block, inbound block

`SimulatedCluster` runs N virtual members in one engine; member ids and addresses are slot
numbers (a member's "address" is its slot).
"""
from __future__ import annotations

import dataclasses
import enum
import re
import math
from collections import defaultdict

import numpy as np

from . import abi


# ------------------------------------------------------------------------------------ configs
@dataclasses.dataclass(frozen=True)
class FailureDetectorConfig:
    """FailureDetectorConfig.java:9-25; presets :29-66."""
    ping_interval: int = 1000
    ping_timeout: int = 500
    ping_req_members: int = 3

    @staticmethod
    def default_config():
        return FailureDetectorConfig()

    @staticmethod
    def default_lan_config():
        return FailureDetectorConfig()

    @staticmethod
    def default_wan_config():
        return FailureDetectorConfig(ping_interval=5000, ping_timeout=3000)

    @staticmethod
    def default_local_config():
        return FailureDetectorConfig(ping_interval=1000, ping_timeout=200, ping_req_members=1)

    def with_(self, **kw):
        return dataclasses.replace(self, **kw)


@dataclasses.dataclass(frozen=True)
class GossipConfig:
    """GossipConfig.java:9-25; presets :29-62."""
    gossip_interval: int = 200
    gossip_fanout: int = 3
    gossip_repeat_mult: int = 3
    gossip_segmentation_threshold: int = 1000

    @staticmethod
    def default_config():
        return GossipConfig()

    @staticmethod
    def default_lan_config():
        return GossipConfig()

    @staticmethod
    def default_wan_config():
        return GossipConfig(gossip_fanout=4)

    @staticmethod
    def default_local_config():
        return GossipConfig(gossip_repeat_mult=2, gossip_interval=100)

    def with_(self, **kw):
        return dataclasses.replace(self, **kw)


@dataclasses.dataclass(frozen=True)
class MembershipConfig:
    """MembershipConfig.java:14-32; presets :36-71."""
    seed_members: tuple = ()
    sync_interval: int = 30000
    sync_timeout: int = 3000
    suspicion_mult: int = 5
    removed_members_history_size: int = 42
    namespace: str = "default"

    @staticmethod
    def default_config():
        return MembershipConfig()

    @staticmethod
    def default_lan_config():
        return MembershipConfig()

    @staticmethod
    def default_wan_config():
        return MembershipConfig(suspicion_mult=6, sync_interval=60000)

    @staticmethod
    def default_local_config():
        return MembershipConfig(suspicion_mult=3, sync_interval=15000)

    def with_(self, **kw):
        return dataclasses.replace(self, **kw)


@dataclasses.dataclass(frozen=True)
class ClusterConfig:
    """ClusterConfig.java:28-93 (knobs on the hot path only)."""
    failure_detector_config: FailureDetectorConfig = FailureDetectorConfig()
    gossip_config: GossipConfig = GossipConfig()
    membership_config: MembershipConfig = MembershipConfig()
    metadata_timeout: int = 3000

    @staticmethod
    def default_config():
        return ClusterConfig()

    @staticmethod
    def default_lan_config():
        return ClusterConfig()

    @staticmethod
    def default_wan_config():
        return ClusterConfig(FailureDetectorConfig.default_wan_config(), GossipConfig.default_wan_config(),
                             MembershipConfig.default_wan_config(), metadata_timeout=10000)

    @staticmethod
    def default_local_config():
        return ClusterConfig(FailureDetectorConfig.default_local_config(), GossipConfig.default_local_config(),
                             MembershipConfig.default_local_config(), metadata_timeout=1000)

    # fluent clone-on-write mutators, as ClusterConfig.failureDetector(op) / gossip(op) / membership(op)
    def failure_detector(self, **kw):
        return dataclasses.replace(self, failure_detector_config=self.failure_detector_config.with_(**kw))

    def gossip(self, **kw):
        return dataclasses.replace(self, gossip_config=self.gossip_config.with_(**kw))

    def membership(self, **kw):
        return dataclasses.replace(self, membership_config=self.membership_config.with_(**kw))

    def with_metadata_timeout(self, ms: int):
        return dataclasses.replace(self, metadata_timeout=ms)

    def to_abi(self, lib, **engine_knobs) -> abi.swim_config:
        fd, g, m = self.failure_detector_config, self.gossip_config, self.membership_config
        return abi.default_config(
            lib, 0, ping_interval=fd.ping_interval, ping_timeout=fd.ping_timeout,
            ping_req_members=fd.ping_req_members, gossip_interval=g.gossip_interval,
            gossip_fanout=g.gossip_fanout, gossip_repeat_mult=g.gossip_repeat_mult,
            gossip_segmentation_threshold=g.gossip_segmentation_threshold,
            sync_interval=m.sync_interval, sync_timeout=m.sync_timeout, suspicion_mult=m.suspicion_mult,
            removed_members_history_size=m.removed_members_history_size,
            metadata_timeout=self.metadata_timeout, **engine_knobs)


# ------------------------------------------------------------------------------------ ClusterMath
class ClusterMath:
    """ClusterMath.java:8-136."""

    @staticmethod
    def ceil_log2(num: int) -> int:  # :133-135, 32 - numberOfLeadingZeros
        return (num & 0xFFFFFFFF).bit_length()

    @staticmethod
    def gossip_convergence_probability(fanout, repeat_mult, cluster_size, loss) -> float:  # :38-43
        fanout_with_loss = (1.0 - loss) * fanout
        spread_size = cluster_size - math.pow(cluster_size, -(fanout_with_loss * repeat_mult - 2))
        return spread_size / cluster_size

    @staticmethod
    def gossip_convergence_percent(fanout, repeat_mult, cluster_size, loss_percent) -> float:  # :23-27
        return ClusterMath.gossip_convergence_probability(fanout, repeat_mult, cluster_size, loss_percent / 100.0) * 100

    @staticmethod
    def max_messages_per_gossip_per_node(fanout, repeat_mult, cluster_size) -> int:  # :65-67
        return fanout * repeat_mult * ClusterMath.ceil_log2(cluster_size)

    @staticmethod
    def max_messages_per_gossip_total(fanout, repeat_mult, cluster_size) -> int:  # :53-55
        return cluster_size * ClusterMath.max_messages_per_gossip_per_node(fanout, repeat_mult, cluster_size)

    @staticmethod
    def gossip_periods_to_spread(repeat_mult, cluster_size) -> int:  # :111-113
        return repeat_mult * ClusterMath.ceil_log2(cluster_size)

    @staticmethod
    def gossip_periods_to_sweep(repeat_mult, cluster_size) -> int:  # :99-102
        return 2 * (ClusterMath.gossip_periods_to_spread(repeat_mult, cluster_size) + 1)

    @staticmethod
    def gossip_dissemination_time(repeat_mult, cluster_size, gossip_interval) -> int:  # :77-79
        return ClusterMath.gossip_periods_to_spread(repeat_mult, cluster_size) * gossip_interval

    @staticmethod
    def gossip_timeout_to_sweep(repeat_mult, cluster_size, gossip_interval) -> int:  # :88-90
        return ClusterMath.gossip_periods_to_sweep(repeat_mult, cluster_size) * gossip_interval

    @staticmethod
    def suspicion_timeout(suspicion_mult, cluster_size, ping_interval) -> int:  # :123-125
        return suspicion_mult * ClusterMath.ceil_log2(cluster_size) * ping_interval


# ------------------------------------------------------------------------------------ members & events
class MemberStatus(enum.IntEnum):  # MemberStatus.java:3-19
    ALIVE = abi.ALIVE
    SUSPECT = abi.SUSPECT
    LEAVING = abi.LEAVING
    DEAD = abi.DEAD


@dataclasses.dataclass(frozen=True)
class Member:  # Member.java:16-143 — id and address are the member's slot
    id: int
    namespace: str = "default"

    @property
    def address(self) -> int:
        return self.id


@dataclasses.dataclass(frozen=True)
class MembershipRecord:  # MembershipRecord.java:20-22
    member: Member
    status: MemberStatus
    incarnation: int


@dataclasses.dataclass(frozen=True)
class MembershipEvent:  # MembershipEvent.java:13-148
    class Type(enum.IntEnum):
        ADDED = abi.EV_ADDED
        REMOVED = abi.EV_REMOVED
        LEAVING = abi.EV_LEAVING
        UPDATED = abi.EV_UPDATED

    type: "MembershipEvent.Type"
    member: Member
    timestamp: int  # virtual milliseconds

    def is_added(self):
        return self.type == MembershipEvent.Type.ADDED

    def is_removed(self):
        return self.type == MembershipEvent.Type.REMOVED

    def is_leaving(self):
        return self.type == MembershipEvent.Type.LEAVING

    def is_updated(self):
        return self.type == MembershipEvent.Type.UPDATED


@dataclasses.dataclass(frozen=True)
class FailureDetectorEvent:  # FailureDetectorEvent.java:8-33
    member: Member
    status: MemberStatus


_FD_EV = {abi.EV_FD_ALIVE: MemberStatus.ALIVE, abi.EV_FD_SUSPECT: MemberStatus.SUSPECT,
          abi.EV_FD_DEAD: MemberStatus.DEAD}


# ------------------------------------------------------------------------------------ views
class MembershipView:
    """MembershipProtocol of one virtual member (MembershipProtocol.java:14-65)."""

    def __init__(self, cluster: "SimulatedCluster", m: int):
        self._c, self._m = cluster, m

    def member(self) -> Member:
        return Member(self._m)

    def _row(self):
        return self._c.engine.read_view(self._m)

    def members(self) -> list[Member]:
        row = self._row()
        return [Member(int(i)) for i in np.nonzero(abi.cell_in_members(row))[0]]

    def other_members(self) -> list[Member]:
        return [x for x in self.members() if x.id != self._m]

    def member_by_id(self, member_id: int):
        row = self._row()
        return Member(member_id) if 0 <= member_id < len(row) and abi.cell_in_members(row[member_id]) else None

    def membership_records(self) -> list[MembershipRecord]:
        row = self._row()
        idx = np.nonzero(abi.cell_in_table(row))[0]
        st, inc = abi.cell_status(row[idx]), abi.cell_inc(row[idx])
        return [MembershipRecord(Member(int(i)), MemberStatus(int(s)), int(n)) for i, s, n in zip(idx, st, inc)]

    def members_by_status(self, status: MemberStatus) -> list[Member]:
        return [r.member for r in self.membership_records() if r.status == status]

    def listen(self) -> list[MembershipEvent]:
        """Events published since the last call (the DirectProcessor stream, drained)."""
        return self._c._take(self._m, fd=False)

    def incarnation(self) -> int:
        return int(abi.cell_inc(self._row()[self._m]))


class FailureDetectorView:
    def __init__(self, cluster: "SimulatedCluster", m: int):
        self._c, self._m = cluster, m

    def listen(self) -> list[FailureDetectorEvent]:
        return self._c._take(self._m, fd=True)


_NAMESPACE_PATTERN = re.compile(r"(\w+[\w\-./]*\w)+", re.ASCII)  # ClusterImpl.java:60, matches()


def validate_namespace(namespace: str) -> None:
    """ClusterImpl.validateConfiguration (:350-353)."""
    if not _NAMESPACE_PATTERN.fullmatch(namespace or ""):
        raise ValueError("Invalid cluster config: membership.namespace format is invalid")


def namespaces_related(ns1: str, ns2: str) -> bool:
    """MembershipProtocolImpl.areNamespacesRelated (:511-536) over java.nio Path name components."""
    a = [x for x in ns1.split("/") if x]
    b = [x for x in ns2.split("/") if x]
    if a == b:
        return True
    if len(a) == len(b):
        return False
    shorter, longer = (a, b) if len(a) < len(b) else (b, a)
    return longer[:len(shorter)] == shorter


class GossipMessage:
    """A user gossip as listen() delivers it (transport-api Message: the data the spreader passed)."""

    def __init__(self, data, gossiper: int):
        self.data = data
        self.gossiper = gossiper

    def __repr__(self):
        return f"GossipMessage(data={self.data!r}, gossiper={self.gossiper})"


class SpreadFuture:
    """The Mono<String> GossipProtocol.spread returns: completes once the gossip has been spread for
    periodsToSpread rounds (GossipProtocolImpl.java:167-180)."""

    def __init__(self):
        self.done = False
        self.completed_ms = None


class GossipProtocolView:
    """GossipProtocol (GossipProtocol.java:12-29) of one virtual member: spread() / listen()."""

    def __init__(self, cluster: "SimulatedCluster", m: int):
        self._c, self._m = cluster, m

    def spread(self, data) -> SpreadFuture:  # GossipProtocolImpl.spread (:126-130)
        pid = self._c._payload_id(data)
        fut = SpreadFuture()
        self._c._futures[(self._m, pid)] = fut
        self._c.engine.spread(self._m, pid)
        return fut

    def listen(self) -> list[GossipMessage]:  # the new gossips this member received since the last call
        self._c._pump()
        out = self._c._gossip_queues[self._m]
        self._c._gossip_queues[self._m] = []
        return out


def _check_loss_percent(loss_percent: int) -> None:
    """OutboundSettings' loss is a percentage (NetworkEmulator.java:349-352)."""
    if not 0 <= int(loss_percent) <= 100:
        raise ValueError(f"loss_percent must be within 0..100: {loss_percent}")


class NetworkEmulator:
    """NetworkEmulator of one member (NetworkEmulator.java): outbound loss and mean delay per
    destination or by default, inbound pass/block per source or by default.  Delays are quantised to
    engine ticks (include/swim_delay.h)."""

    def __init__(self, cluster: "SimulatedCluster", m: int):
        self._c, self._m = cluster, m

    # a refused setting changes nothing: the loss is range-checked first and the delay (which the
    # engine refuses above its tick cap) is set before the loss
    def outbound_settings(self, destination: int, loss_percent: int, mean_delay: int = 0):  # :69-73
        _check_loss_percent(loss_percent)
        self._c.engine.set_link_delay(self._m, destination, mean_delay)
        self._c._note_link(self._m, destination)
        self._c.engine.set_link_loss(self._m, destination, loss_percent)

    def set_default_outbound_settings(self, loss_percent: int, mean_delay: int = 0):  # :80-83
        _check_loss_percent(loss_percent)
        self._c.engine.set_default_delay(mean_delay, self._m)
        self._c.engine.set_default_loss(loss_percent, self._m)

    def block_all_outbound(self):  # :86-90
        for d in self._c._links_from(self._m):
            self._c.engine.set_link_loss(self._m, d, -1)
            self._c.engine.set_link_delay(self._m, d, -1)
        self._c.engine.set_default_loss(100, self._m)
        self._c.engine.set_default_delay(0, self._m)

    def unblock_all_outbound(self):  # :93-97
        for d in self._c._links_from(self._m):
            self._c.engine.set_link_loss(self._m, d, -1)
            self._c.engine.set_link_delay(self._m, d, -1)
        self._c.engine.set_default_loss(0, self._m)
        self._c.engine.set_default_delay(0, self._m)

    def block_outbound(self, *destinations):  # :110-121
        for d in _flatten(destinations):
            self._c._note_link(self._m, d)
            self._c.engine.set_link_loss(self._m, d, 100)
            self._c.engine.set_link_delay(self._m, d, 0)

    def unblock_outbound(self, *destinations):  # :128-139
        for d in _flatten(destinations):
            self._c.engine.set_link_loss(self._m, d, -1)
            self._c.engine.set_link_delay(self._m, d, -1)

    def inbound_settings(self, destination: int, shall_pass: bool):  # :221-225
        self._c._note_inlink(self._m, destination)
        self._c.engine.set_link_inbound(self._m, destination, 1 if shall_pass else 0)

    def set_default_inbound_settings(self, shall_pass: bool):  # :230-233
        self._c.engine.set_default_inbound(shall_pass, self._m)

    def block_all_inbound(self):  # :236-240
        for s in self._c._inlinks_to(self._m):
            self._c.engine.set_link_inbound(self._m, s, -1)
        self._c.engine.set_default_inbound(False, self._m)

    def unblock_all_inbound(self):  # :243-247
        for s in self._c._inlinks_to(self._m):
            self._c.engine.set_link_inbound(self._m, s, -1)
        self._c.engine.set_default_inbound(True, self._m)

    def block_inbound(self, *sources):  # :260-289
        for s in _flatten(sources):
            self._c._note_inlink(self._m, s)
            self._c.engine.set_link_inbound(self._m, s, 0)

    def unblock_inbound(self, *sources):
        for s in _flatten(sources):
            self._c.engine.set_link_inbound(self._m, s, -1)


def _flatten(xs):
    out = []
    for x in xs:
        if isinstance(x, (list, tuple, set)):
            out.extend(_flatten(x))
        else:
            out.append(int(x.id) if isinstance(x, Member) else int(x))
    return out


# ------------------------------------------------------------------------------------ cluster
class SimulatedCluster:
    """N virtual scalecube-cluster members advancing in lockstep on one MI355X.

    Replaces the per-member `new FailureDetectorImpl / GossipProtocolImpl / MembershipProtocolImpl`
    of ClusterImpl.doStart0 (ClusterImpl.java:260-291) for all members at once.
    """

    def __init__(self, config: ClusterConfig | None = None, size: int = 3, capacity: int | None = None,
                 seed: int = 1, record_fd_events: bool = False, sync_stagger: bool = True, **engine_knobs):
        from . import load_library  # the product path binds libswimgpu.so only
        self.config = config or ClusterConfig.default_config()
        lib = load_library()
        cfg = self.config.to_abi(lib, record_fd_events=int(record_fd_events), sync_stagger=int(sync_stagger),
                                 **engine_knobs)
        self._init(abi.Engine(lib, cfg, capacity or size, size, seed))

    @classmethod
    def from_engine(cls, engine: abi.Engine, config: ClusterConfig | None = None) -> "SimulatedCluster":
        """Wrap an existing engine handle (any library exporting include/swim.h)."""
        self = cls.__new__(cls)
        self.config = config or ClusterConfig.default_config()
        self._init(engine)
        return self

    def _init(self, engine: abi.Engine):
        self.engine = engine
        self._queues = defaultdict(list)
        self._fd_queues = defaultdict(list)
        self._links = defaultdict(set)
        self._inlinks = defaultdict(set)
        self._gossip_queues = defaultdict(list)
        self._payloads = []      # payload handle -> the spread data
        self._futures = {}       # (member, payload handle) -> SpreadFuture
        _, self.tick_ms, self.ticks_per_period = engine.now()
        seeds = list(self.config.membership_config.seed_members)
        if seeds:
            engine.set_seeds(seeds)

    # -- time
    def step(self, periods: int = 1):
        self.engine.step(periods)
        self._pump()

    def step_ticks(self, ticks: int = 1):
        self.engine.step_ticks(ticks)
        self._pump()

    def await_seconds(self, seconds: float):
        """BaseTest.awaitSeconds (cluster/src/test/.../BaseTest.java:33-39) in virtual time."""
        self.step_ticks(int(round(seconds * 1000 / self.tick_ms)))

    def await_suspicion(self, cluster_size: int):
        """BaseTest.awaitSuspicion (:41-47): suspicion timeout + 2 s of virtual time."""
        m = self.config.membership_config
        fd = self.config.failure_detector_config
        ms = ClusterMath.suspicion_timeout(m.suspicion_mult, cluster_size, fd.ping_interval)
        self.await_seconds(ms // 1000 + 2)

    @property
    def now_ms(self) -> int:
        return self.engine.now()[0] * self.tick_ms

    # -- lifecycle
    def kill(self, m: int):
        self.engine.kill(m)

    def shutdown(self, m: int):
        """ClusterImpl.shutdown (:508-517): leaveCluster, then stop once the LEAVING gossip spread."""
        self.engine.leave(m, True)

    def leave_cluster(self, m: int):
        """MembershipProtocolImpl.leaveCluster (:233-242) without stopping the member."""
        self.engine.leave(m, False)

    def join(self, m: int, same_address_as: int = None, config: "ClusterConfig | None" = None):
        """Start member m; with same_address_as, on that stopped member's address (a restart on the
        same port, MembershipProtocolTest.testRestartStoppedMembersOnSameAddresses :654-711); with
        config, member m's own ClusterConfig: its membershipConfig().seedMembers() become m's seed
        list (MembershipProtocolImpl :120-130, cleanUpSeedMembers :171-190)."""
        if config is not None:
            self.set_member_config(m, config)
        if same_address_as is None:
            self.engine.join(m)
        else:
            self.engine.join_at(m, same_address_as)

    def set_member_config(self, m: int, config: "ClusterConfig"):
        """Member m's own ClusterConfig, as far as the protocol layer reads it per member: its seed
        members (start0's initial SYNCs, selectSyncAddress); the timing knobs are engine-wide."""
        self.engine.set_member_seeds(m, _flatten(config.membership_config.seed_members))

    # -- views
    def membership(self, m: int) -> MembershipView:
        return MembershipView(self, m)

    def failure_detector(self, m: int) -> FailureDetectorView:
        return FailureDetectorView(self, m)

    def gossip(self, m: int) -> GossipProtocolView:
        return GossipProtocolView(self, m)

    def network_emulator(self, m: int) -> NetworkEmulator:
        return NetworkEmulator(self, m)

    def update_metadata(self, m: int):
        """ClusterImpl.updateMetadata (:497-500) of member m (a new metadata version)."""
        self.engine.update_metadata(m)

    def set_namespaces(self, namespaces):
        """MembershipConfig.namespace of every member (capacity strings), validated as the reference
        does; members of unrelated namespaces never enter each other's tables."""
        names = sorted(set(namespaces))
        for x in names:
            validate_namespace(x)
        gid = {x: i for i, x in enumerate(names)}
        rel = np.array([[namespaces_related(x, y) for y in names] for x in names], dtype=np.uint8)
        self.engine.set_namespaces(np.array([gid[x] for x in namespaces], dtype=np.uint16), rel)

    def partition(self, groups):
        self.engine.set_partition(groups)

    def heal(self):
        self.engine.set_partition(None)

    # -- internals
    def _note_link(self, a, b):
        self._links[a].add(b)

    def _note_inlink(self, a, b):
        self._inlinks[a].add(b)

    def _links_from(self, a):  # ascending, as SimulatedCluster.takeOutLinks (TreeSet)
        s = sorted(self._links[a])
        self._links[a].clear()
        return s

    def _inlinks_to(self, a):
        s = sorted(self._inlinks[a])
        self._inlinks[a].clear()
        return s

    def _payload_id(self, data) -> int:
        self._payloads.append(data)
        return len(self._payloads) - 1

    def _pump(self):
        ev = self.engine.drain_events()
        for e in ev:
            t = int(e["type"])
            if t == abi.EV_GOSSIP:
                self._gossip_queues[int(e["viewer"])].append(
                    GossipMessage(self._payloads[int(e["data"])], int(e["subject"])))
            elif t == abi.EV_SPREAD_DONE:
                fut = self._futures.pop((int(e["viewer"]), int(e["data"])), None)
                if fut is not None:
                    fut.done = True
                    fut.completed_ms = int(e["tick"]) * self.tick_ms
            elif t in _FD_EV:
                self._fd_queues[int(e["viewer"])].append(FailureDetectorEvent(Member(int(e["subject"])), _FD_EV[t]))
            else:
                self._queues[int(e["viewer"])].append(
                    MembershipEvent(MembershipEvent.Type(t), Member(int(e["subject"])), int(e["tick"]) * self.tick_ms))

    def _take(self, m: int, fd: bool):
        self._pump()
        q = self._fd_queues if fd else self._queues
        out = q[m]
        q[m] = []
        return out
