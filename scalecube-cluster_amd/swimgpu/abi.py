"""ctypes mirror of include/swim.h (the engine's C ABI).

`bind(lib)` declares every prototype on a loaded CDLL.  `Engine` is a thin, typed wrapper over
one `swim_engine*` handle; it is backend-agnostic (it only needs a library exporting the ABI),
which is what lets the parity tests drive the CPU oracle and the GPU engine through one code path.
The product entry point (`swimgpu.SimulatedCluster`) always binds libswimgpu.so.
"""
from __future__ import annotations

import ctypes as C
from ctypes import POINTER, byref

import numpy as np

SWIM_OK = 0
SWIM_EINVAL = -1
SWIM_ENOMEM = -2
SWIM_EDEVICE = -3
SWIM_ECAPACITY = -4
SWIM_ESTATE = -5
_ERRORS = {
    SWIM_EINVAL: "SWIM_EINVAL (bad argument / unsupported configuration)",
    SWIM_ENOMEM: "SWIM_ENOMEM (allocation failed)",
    SWIM_EDEVICE: "SWIM_EDEVICE (HIP runtime error)",
    SWIM_ECAPACITY: "SWIM_ECAPACITY (fixed-capacity structure overflowed)",
    SWIM_ESTATE: "SWIM_ESTATE (invalid in the member's current state)",
}

ALIVE, SUSPECT, LEAVING, DEAD = 0, 1, 2, 3
EV_ADDED, EV_REMOVED, EV_LEAVING, EV_UPDATED = 0, 1, 2, 3
EV_GOSSIP, EV_SPREAD_DONE = 32, 33  # user gossips (swim_spread)
GOSSIP_USER, GOSSIP_USER_SPREAD = 4, 5  # swim_gossip.status of a user gossip
EV_FD_ALIVE, EV_FD_SUSPECT, EV_FD_DEAD = 16, 17, 18
PHASE_TIMERS, PHASE_FD, PHASE_GOSSIP, PHASE_SYNC, PHASE_SYNCACK, PHASE_CONTROL = 1, 2, 3, 4, 5, 6
ALL_MEMBERS = 0xFFFFFFFF


class SwimError(RuntimeError):
    def __init__(self, fn: str, code: int):
        super().__init__(f"{fn} failed: {_ERRORS.get(code, code)}")
        self.code = code


class swim_config(C.Structure):
    _fields_ = [
        ("ping_interval", C.c_int32),
        ("ping_timeout", C.c_int32),
        ("ping_req_members", C.c_int32),
        ("gossip_interval", C.c_int32),
        ("gossip_fanout", C.c_int32),
        ("gossip_repeat_mult", C.c_int32),
        ("gossip_segmentation_threshold", C.c_int32),
        ("sync_interval", C.c_int32),
        ("sync_timeout", C.c_int32),
        ("suspicion_mult", C.c_int32),
        ("removed_members_history_size", C.c_int32),
        ("metadata_timeout", C.c_int32),
        ("tick_ms", C.c_int32),
        ("sync_stagger", C.c_int32),
        ("record_fd_events", C.c_int32),
        ("gossip_capacity", C.c_uint32),
        ("collector_capacity", C.c_uint32),
        ("event_capacity", C.c_uint32),
        ("device", C.c_int32),
        ("local_shards", C.c_int32),
        ("timer_stagger", C.c_int32),
        ("timer_capacity", C.c_uint32),
        ("message_capacity", C.c_uint32),
        ("interval_capacity", C.c_uint32),
        ("deliver_wave_min", C.c_uint32),
        ("delay_capacity", C.c_uint32),
        ("timer_pool_capacity", C.c_uint32),
    ]


class swim_event(C.Structure):
    _fields_ = [
        ("tick", C.c_uint64),
        ("viewer", C.c_uint32),
        ("subject", C.c_uint32),
        ("type", C.c_uint32),
        ("phase", C.c_uint32),
        ("minor", C.c_uint32),
        ("data", C.c_uint32),
    ]


EVENT_DTYPE = np.dtype(
    [("tick", "<u8"), ("viewer", "<u4"), ("subject", "<u4"), ("type", "<u4"), ("phase", "<u4"),
     ("minor", "<u4"), ("data", "<u4")])


class swim_stats(C.Structure):
    _fields_ = [(name, C.c_uint64) for name in (
        "ticks", "pings", "ping_reqs", "fd_events", "gossips_created", "gossip_messages",
        "gossip_accepted", "syncs", "sync_acks", "sync_records", "fetches", "fetch_ok",
        "timers_fired", "events", "capacity_errors")] + [
        ("gossips_by_reason", C.c_uint64 * 7), ("reserved", C.c_uint64 * 2)]

# swim_stats.gossips_by_reason indices (SWIM_ORIG_*, swim.h)
ORIG_REASONS = ("fd", "sync", "refute", "leaving", "leave", "metadata", "user")


class swim_member_state(C.Structure):
    _fields_ = [
        ("up", C.c_uint8),
        ("joined", C.c_uint8),
        ("leave_pending", C.c_uint8),
        ("join_pending", C.c_uint8),
        ("remote_idx", C.c_int32),
        ("fd_period", C.c_uint64),
        ("ping_cursor", C.c_uint32),
        ("ping_len", C.c_uint32),
        ("remote_len", C.c_uint32),
        ("gossip_len", C.c_uint32),
        ("gossip_period", C.c_uint64),
        ("gossip_counter", C.c_uint64),
        ("table_size", C.c_uint32),
        ("members_size", C.c_uint32),
        ("fd_start", C.c_int64),
        ("gossip_start", C.c_int64),
        ("sync_start", C.c_int64),
        ("sync_on", C.c_uint8),
        ("pad", C.c_uint8 * 3),
        ("ack_target", C.c_uint32),
        ("ack_due", C.c_uint64),
        ("relay_target", C.c_uint32),
        ("relay_pending", C.c_uint32),
        ("relay_due", C.c_uint64),
        ("leave_gossiper", C.c_uint32),
        ("pending_acks", C.c_uint32),
        ("leave_seq", C.c_uint64),
    ]


class swim_gossip(C.Structure):
    _fields_ = [
        ("gossiper", C.c_uint32),
        ("subject", C.c_uint32),
        ("seq", C.c_uint64),
        ("inc", C.c_int32),
        ("status", C.c_uint32),
        ("infection_period", C.c_uint64),
        ("infected", C.c_uint32 * 2),
    ]


GOSSIP_DTYPE = np.dtype(
    [("gossiper", "<u4"), ("subject", "<u4"), ("seq", "<u8"), ("inc", "<i4"), ("status", "<u4"),
     ("infection_period", "<u8"), ("infected", "<u4", (2,))])


class swim_interval(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("hi", C.c_uint64)]


class swim_record(C.Structure):
    _fields_ = [("member", C.c_uint32), ("status", C.c_uint32), ("inc", C.c_int32), ("pad", C.c_uint32)]


RECORD_DTYPE = np.dtype([("member", "<u4"), ("status", "<u4"), ("inc", "<i4"), ("pad", "<u4")])


class swim_quiet_stats(C.Structure):
    _fields_ = [("ticks", C.c_uint64), ("windows", C.c_uint64), ("attempts", C.c_uint64), ("cut_short", C.c_uint64),
                ("precomputed", C.c_uint64)]


class swim_kernel_profile(C.Structure):
    _fields_ = [("launches", C.c_uint64), ("total_ms", C.c_double), ("messages", C.c_uint64),
                ("records", C.c_uint64), ("alg_bytes", C.c_uint64), ("examined", C.c_uint64)]


_u32p = POINTER(C.c_uint32)
_u64p = POINTER(C.c_uint64)
_engp = C.c_void_p

PROTOTYPES = {
    "swim_config_default": (C.c_int32, [POINTER(swim_config), C.c_int32]),
    "swim_ceil_log2": (C.c_int32, [C.c_int32]),
    "swim_gossip_periods_to_spread": (C.c_int32, [C.c_int32, C.c_int32]),
    "swim_gossip_periods_to_sweep": (C.c_int32, [C.c_int32, C.c_int32]),
    "swim_suspicion_timeout": (C.c_int64, [C.c_int32, C.c_int32, C.c_int64]),
    "swim_create": (C.c_int32, [POINTER(swim_config), C.c_uint32, C.c_uint32, C.c_uint64, POINTER(_engp)]),
    "swim_destroy": (C.c_int32, [_engp]),
    "swim_comm_unique_id": (C.c_int32, [POINTER(C.c_uint8)]),
    "swim_create_shard": (C.c_int32, [POINTER(swim_config), C.c_uint32, C.c_uint32, C.c_uint64, C.c_int32, C.c_int32,
                                      POINTER(C.c_uint8), POINTER(_engp)]),
    "swim_shard_info": (C.c_int32, [_engp, POINTER(C.c_int32), POINTER(C.c_int32), _u32p, _u32p]),
    "swim_exchange_info": (C.c_int32, [_engp, _u32p]),
    "swim_step_ticks": (C.c_int32, [_engp, C.c_uint32]),
    "swim_step": (C.c_int32, [_engp, C.c_uint32]),
    "swim_now": (C.c_int32, [_engp, _u64p, _u32p, _u32p]),
    "swim_set_seeds": (C.c_int32, [_engp, _u32p, C.c_uint32]),
    "swim_set_member_seeds": (C.c_int32, [_engp, C.c_uint32, _u32p, C.c_uint32]),
    "swim_kill": (C.c_int32, [_engp, C.c_uint32]),
    "swim_leave": (C.c_int32, [_engp, C.c_uint32, C.c_int32]),
    "swim_spread": (C.c_int32, [_engp, C.c_uint32, C.c_uint32]),
    "swim_update_metadata": (C.c_int32, [_engp, C.c_uint32]),
    "swim_set_namespaces": (C.c_int32, [_engp, C.c_void_p, C.c_uint32, C.c_void_p]),
    "swim_join": (C.c_int32, [_engp, C.c_uint32]),
    "swim_join_at": (C.c_int32, [_engp, C.c_uint32, C.c_uint32]),
    "swim_set_default_loss": (C.c_int32, [_engp, C.c_uint32, C.c_int32]),
    "swim_set_link_loss": (C.c_int32, [_engp, C.c_uint32, C.c_uint32, C.c_int32]),
    "swim_set_default_delay": (C.c_int32, [_engp, C.c_uint32, C.c_int32]),
    "swim_set_link_delay": (C.c_int32, [_engp, C.c_uint32, C.c_uint32, C.c_int32]),
    "swim_set_link_inbound": (C.c_int32, [_engp, C.c_uint32, C.c_uint32, C.c_int32]),
    "swim_set_default_inbound": (C.c_int32, [_engp, C.c_uint32, C.c_int32]),
    "swim_set_partition": (C.c_int32, [_engp, POINTER(C.c_uint16)]),
    "swim_read_view": (C.c_int32, [_engp, C.c_uint32, _u64p]),
    "swim_drain_events": (C.c_int32, [_engp, POINTER(swim_event), C.c_size_t, POINTER(C.c_size_t)]),
    "swim_get_stats": (C.c_int32, [_engp, POINTER(swim_stats)]),
    "swim_read_member": (C.c_int32, [_engp, C.c_uint32, POINTER(swim_member_state)]),
    "swim_read_ping_list": (C.c_int32, [_engp, C.c_uint32, _u32p, C.c_uint32, _u32p]),
    "swim_read_remote_list": (C.c_int32, [_engp, C.c_uint32, _u32p, C.c_uint32, _u32p]),
    "swim_read_gossips": (C.c_int32, [_engp, C.c_uint32, POINTER(swim_gossip), C.c_uint32, _u32p]),
    "swim_read_collector": (C.c_int32, [_engp, C.c_uint32, C.c_uint32, POINTER(swim_interval), C.c_uint32, _u32p]),
    "swim_profile_enable": (C.c_int32, [_engp, C.c_int32]),
    "swim_profile_merge": (C.c_int32, [_engp, POINTER(swim_kernel_profile)]),
    "swim_profile_fanout": (C.c_int32, [_engp, POINTER(swim_kernel_profile)]),
    "swim_profile_deliver": (C.c_int32, [_engp, POINTER(swim_kernel_profile)]),
    "swim_profile_quiet": (C.c_int32, [_engp, POINTER(swim_kernel_profile)]),
    "swim_ingest_sync": (C.c_int32, [_engp, C.c_uint32, POINTER(swim_record), C.c_uint32, C.c_int32]),
    "swim_set_quiet_path": (C.c_int32, [_engp, C.c_int32]),
    "swim_debug_counters": (C.c_int32, [_u64p, C.c_uint32, C.c_int32]),
    "swim_get_quiet_stats": (C.c_int32, [_engp, POINTER(swim_quiet_stats)]),
    "swim_philox": (C.c_int32, [_u32p, _u32p, _u32p]),
    "swim_kat_overrides": (C.c_int32, [POINTER(C.c_int32), C.c_uint32, POINTER(C.c_uint8)]),
    "swim_kat_collector": (C.c_int32, [POINTER(C.c_uint8), POINTER(C.c_int64), C.c_uint32, POINTER(C.c_int64)]),
}


def bind(lib: C.CDLL) -> C.CDLL:
    """Declare every swim.h prototype on `lib`; raises AttributeError if a symbol is missing."""
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def _check(fn: str, rc: int) -> None:
    if rc != SWIM_OK:
        raise SwimError(fn, rc)


def default_config(lib: C.CDLL, preset: int = 0, **overrides) -> swim_config:
    cfg = swim_config()
    _check("swim_config_default", lib.swim_config_default(byref(cfg), preset))
    for k, v in overrides.items():
        if not hasattr(cfg, k):
            raise AttributeError(f"swim_config has no field {k!r}")
        setattr(cfg, k, v)
    return cfg


COMM_ID_BYTES = 128


def comm_unique_id(lib: C.CDLL) -> bytes:
    """swim_comm_unique_id: rank 0 creates the RCCL bootstrap id the other ranks join with."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    _check("swim_comm_unique_id", lib.swim_comm_unique_id(buf))
    return bytes(buf)


class Engine:
    """One engine handle over any library exporting the swim.h ABI.

    With `world > 1` the handle is rank `rank`'s shard of a multi-process cluster
    (swim_create_shard; every call is collective across the ranks, see swim.h)."""

    def __init__(self, lib: C.CDLL, cfg: swim_config, capacity: int, n_initial: int, seed: int,
                 rank: int = 0, world: int = 1, comm_id: bytes | None = None):
        self.lib = lib
        self.cfg = cfg
        self.capacity = int(capacity)
        h = _engp()
        if world > 1 or comm_id is not None:  # (world 1 with an id: an RCCL engine of one rank)
            if comm_id is None or len(comm_id) != COMM_ID_BYTES:
                raise ValueError("a sharded engine needs the 128-byte id from comm_unique_id() on rank 0")
            cid = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(comm_id)
            _check("swim_create_shard", lib.swim_create_shard(byref(cfg), capacity, n_initial, seed, rank, world,
                                                              cid, byref(h)))
        else:
            _check("swim_create", lib.swim_create(byref(cfg), capacity, n_initial, seed, byref(h)))
        self._h = h

    def shard_info(self) -> dict:
        r, w, lo, cnt = C.c_int32(), C.c_int32(), C.c_uint32(), C.c_uint32()
        _check("swim_shard_info", self.lib.swim_shard_info(self._h, byref(r), byref(w), byref(lo), byref(cnt)))
        return {"rank": r.value, "world": w.value, "lo": lo.value, "count": cnt.value}

    def exchange_info(self) -> dict:
        """swim_exchange_info: how the exchange is set up (which branch of the RCCL setup ran)"""
        f = C.c_uint32()
        _check("swim_exchange_info", self.lib.swim_exchange_info(self._h, byref(f)))
        v = f.value
        return {"flags": v, "exchange": bool(v & 1), "rccl": bool(v & 2), "uncached": bool(v & 4),
                "ipc": bool(v & 8), "ipc_fallback_cached": bool(v & 16)}

    # -- lifecycle ------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.swim_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def step(self, periods: int = 1) -> None:
        self._check_step("swim_step", self.lib.swim_step(self._h, periods))

    def step_ticks(self, ticks: int = 1) -> None:
        self._check_step("swim_step_ticks", self.lib.swim_step_ticks(self._h, ticks))

    def _check_step(self, fn: str, rc: int) -> None:
        if rc == SWIM_ECAPACITY:  # name the structure that overflowed (swim_stats.capacity_errors)
            raise SwimError(f"{fn} (capacity error bits {self.stats()['capacity_errors']:#x})", rc)
        _check(fn, rc)

    def now(self) -> tuple[int, int, int]:
        t, ms, tpp = C.c_uint64(), C.c_uint32(), C.c_uint32()
        _check("swim_now", self.lib.swim_now(self._h, byref(t), byref(ms), byref(tpp)))
        return t.value, ms.value, tpp.value

    # -- control --------------------------------------------------------------------------
    def set_seeds(self, seeds) -> None:
        arr = (C.c_uint32 * len(seeds))(*seeds)
        _check("swim_set_seeds", self.lib.swim_set_seeds(self._h, arr, len(seeds)))

    def set_member_seeds(self, m: int, seeds) -> None:
        """swim_set_member_seeds: member m's own seedMembers (None: back on the engine-wide list)."""
        if seeds is None:
            rc = self.lib.swim_set_member_seeds(self._h, m, None, 0xffffffff)
        else:
            arr = (C.c_uint32 * max(1, len(seeds)))(*seeds)
            rc = self.lib.swim_set_member_seeds(self._h, m, arr, len(seeds))
        _check("swim_set_member_seeds", rc)

    def kill(self, m: int) -> None:
        _check("swim_kill", self.lib.swim_kill(self._h, m))

    def leave(self, m: int, stop_after: bool = True) -> None:
        _check("swim_leave", self.lib.swim_leave(self._h, m, 1 if stop_after else 0))

    def spread(self, m: int, payload: int) -> None:
        """GossipProtocol.spread: a user gossip with a 32-bit payload handle from member m, now."""
        _check("swim_spread", self.lib.swim_spread(self._h, m, payload))

    def update_metadata(self, m: int) -> None:
        """ClusterImpl.updateMetadata: m's metadata changes, ALIVE inc+1 is gossiped."""
        _check("swim_update_metadata", self.lib.swim_update_metadata(self._h, m))

    def set_namespaces(self, ns_of_member, related) -> None:
        """Namespace group per member (uint16[capacity]) + the groups' relation matrix; None: one namespace."""
        if ns_of_member is None:
            _check("swim_set_namespaces", self.lib.swim_set_namespaces(self._h, None, 0, None))
            return
        g = np.ascontiguousarray(ns_of_member, dtype=np.uint16)
        r = np.ascontiguousarray(related, dtype=np.uint8)
        _check("swim_set_namespaces", self.lib.swim_set_namespaces(self._h, g.ctypes.data, int(r.shape[0]), r.ctypes.data))

    def join(self, m: int) -> None:
        _check("swim_join", self.lib.swim_join(self._h, m))

    def join_at(self, m: int, addr_of: int) -> None:
        """Start member m on the address of stopped member addr_of (a restart on the same port)."""
        _check("swim_join_at", self.lib.swim_join_at(self._h, m, addr_of))

    def set_default_loss(self, loss_percent: int, m: int = ALL_MEMBERS) -> None:
        _check("swim_set_default_loss", self.lib.swim_set_default_loss(self._h, m, loss_percent))

    def set_link_loss(self, src: int, dst: int, loss_percent: int) -> None:
        _check("swim_set_link_loss", self.lib.swim_set_link_loss(self._h, src, dst, loss_percent))

    def set_default_delay(self, mean_ms: int, m: int = ALL_MEMBERS) -> None:
        _check("swim_set_default_delay", self.lib.swim_set_default_delay(self._h, m, mean_ms))

    def set_link_delay(self, src: int, dst: int, mean_ms: int) -> None:
        _check("swim_set_link_delay", self.lib.swim_set_link_delay(self._h, src, dst, mean_ms))

    def set_link_inbound(self, dst: int, src: int, shall_pass: int) -> None:
        _check("swim_set_link_inbound", self.lib.swim_set_link_inbound(self._h, dst, src, shall_pass))

    def set_default_inbound(self, shall_pass: bool, m: int = ALL_MEMBERS) -> None:
        _check("swim_set_default_inbound", self.lib.swim_set_default_inbound(self._h, m, 1 if shall_pass else 0))

    def set_partition(self, groups) -> None:
        if groups is None:
            _check("swim_set_partition", self.lib.swim_set_partition(self._h, None))
            return
        g = np.ascontiguousarray(groups, dtype=np.uint16)
        assert g.shape == (self.capacity,)
        _check("swim_set_partition", self.lib.swim_set_partition(self._h, g.ctypes.data_as(POINTER(C.c_uint16))))

    # -- readback -------------------------------------------------------------------------
    def read_view(self, viewer: int) -> np.ndarray:
        out = np.empty(self.capacity, dtype=np.uint64)
        _check("swim_read_view", self.lib.swim_read_view(self._h, viewer, out.ctypes.data_as(_u64p)))
        return out

    def drain_events(self, cap: int = 1 << 20) -> np.ndarray:
        chunks = []
        while True:
            buf = np.zeros(cap, dtype=EVENT_DTYPE)
            n = C.c_size_t()
            _check("swim_drain_events", self.lib.swim_drain_events(
                self._h, buf.ctypes.data_as(POINTER(swim_event)), cap, byref(n)))
            chunks.append(buf[: n.value])
            if n.value < cap:
                break
        return np.concatenate(chunks) if chunks else np.zeros(0, dtype=EVENT_DTYPE)

    def stats(self) -> dict:
        s = swim_stats()
        _check("swim_get_stats", self.lib.swim_get_stats(self._h, byref(s)))
        out = {name: getattr(s, name) for name, _ in swim_stats._fields_
               if name not in ("reserved", "gossips_by_reason")}
        # gossips_created split by origination reason: orig_fd, orig_sync, ... (SWIM_ORIG_*)
        out.update({f"orig_{r}": int(s.gossips_by_reason[i]) for i, r in enumerate(ORIG_REASONS)})
        return out

    def read_member(self, m: int) -> dict:
        s = swim_member_state()
        _check("swim_read_member", self.lib.swim_read_member(self._h, m, byref(s)))
        return {name: getattr(s, name) for name, _ in swim_member_state._fields_ if not name.startswith("pad")}

    def _read_list(self, fn: str, m: int) -> np.ndarray:
        ln = C.c_uint32()
        _check(fn, getattr(self.lib, fn)(self._h, m, None, 0, byref(ln)))
        out = np.empty(ln.value, dtype=np.uint32)
        if ln.value:
            _check(fn, getattr(self.lib, fn)(self._h, m, out.ctypes.data_as(_u32p), ln.value, byref(ln)))
        return out

    def read_ping_list(self, m: int) -> np.ndarray:
        return self._read_list("swim_read_ping_list", m)

    def read_remote_list(self, m: int) -> np.ndarray:
        return self._read_list("swim_read_remote_list", m)

    def read_gossips(self, m: int) -> np.ndarray:
        ln = C.c_uint32()
        _check("swim_read_gossips", self.lib.swim_read_gossips(self._h, m, None, 0, byref(ln)))
        out = np.zeros(ln.value, dtype=GOSSIP_DTYPE)
        if ln.value:
            _check("swim_read_gossips", self.lib.swim_read_gossips(
                self._h, m, out.ctypes.data_as(POINTER(swim_gossip)), ln.value, byref(ln)))
        return out

    def profile_enable(self, on: bool = True) -> None:
        _check("swim_profile_enable", self.lib.swim_profile_enable(self._h, 1 if on else 0))

    def profile_merge(self) -> dict:
        p = swim_kernel_profile()
        _check("swim_profile_merge", self.lib.swim_profile_merge(self._h, byref(p)))
        return {name: getattr(p, name) for name, _ in swim_kernel_profile._fields_}

    def profile_fanout(self) -> dict:
        """Sampled timing of the gossip fanout kernel (k_gossip_emit), see swim.h."""
        p = swim_kernel_profile()
        _check("swim_profile_fanout", self.lib.swim_profile_fanout(self._h, byref(p)))
        return {name: getattr(p, name) for name, _ in swim_kernel_profile._fields_}

    def profile_deliver(self) -> dict:
        """Sampled timing of the gossip delivery kernel (k_gossip_deliver), see swim.h."""
        p = swim_kernel_profile()
        _check("swim_profile_deliver", self.lib.swim_profile_deliver(self._h, byref(p)))
        return {name: getattr(p, name) for name, _ in swim_kernel_profile._fields_}

    def ingest_sync(self, viewer: int, records, initial: bool = False) -> None:
        """swim_ingest_sync: onSyncAck at `viewer` for externally supplied (member, status, inc) records,
        in the given order (e.g. swimgpu.wire.engine_records of a decoded SYNC / SYNC_ACK)."""
        arr = np.zeros(len(records), dtype=RECORD_DTYPE)
        for i, (m, st, inc) in enumerate(records):
            arr[i] = (m, st, inc, 0)
        _check("swim_ingest_sync", self.lib.swim_ingest_sync(
            self._h, viewer, arr.ctypes.data_as(POINTER(swim_record)), len(arr), 1 if initial else 0))

    def set_quiet_path(self, enable: bool) -> None:
        """swim_set_quiet_path: quiet windows on (default) or the per-tick kernel chain only."""
        _check("swim_set_quiet_path", self.lib.swim_set_quiet_path(self._h, 1 if enable else 0))

    def quiet_stats(self) -> dict:
        q = swim_quiet_stats()
        _check("swim_get_quiet_stats", self.lib.swim_get_quiet_stats(self._h, byref(q)))
        return {name: getattr(q, name) for name, _ in swim_quiet_stats._fields_}

    def profile_quiet(self) -> dict:
        """HIP-event timing of the quiet windows' kernels (k_quiet_scan .. k_quiet_apply), see swim.h."""
        p = swim_kernel_profile()
        _check("swim_profile_quiet", self.lib.swim_profile_quiet(self._h, byref(p)))
        return {name: getattr(p, name) for name, _ in swim_kernel_profile._fields_}

    def read_collector(self, m: int, gossiper: int) -> list[tuple[int, int]]:
        ln = C.c_uint32()
        _check("swim_read_collector", self.lib.swim_read_collector(self._h, m, gossiper, None, 0, byref(ln)))
        if ln.value == 0:
            return []
        out = (swim_interval * ln.value)()
        _check("swim_read_collector", self.lib.swim_read_collector(self._h, m, gossiper, out, ln.value, byref(ln)))
        return [(x.lo, x.hi) for x in out]


def philox(lib, ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    _check("swim_philox", lib.swim_philox(c, k, o))
    return list(o)


def kat_overrides(lib, cases) -> list[bool]:
    """cases: iterable of (r1_status, r1_inc, r0) with r0 = None or (status, inc)."""
    flat = []
    for r1s, r1i, r0 in cases:
        flat += [r1s, r1i, 0, 0, 0] if r0 is None else [r1s, r1i, 1, r0[0], r0[1]]
    n = len(flat) // 5
    arr = (C.c_int32 * len(flat))(*flat)
    out = (C.c_uint8 * n)()
    _check("swim_kat_overrides", lib.swim_kat_overrides(arr, n, out))
    return [bool(x) for x in out]


def kat_collector(lib, ops) -> list[int]:
    """ops: list of ("add"|"contains"|"size"|"clear", value)."""
    codes = {"add": 0, "contains": 1, "size": 2, "clear": 3}
    n = len(ops)
    kinds = (C.c_uint8 * n)(*[codes[o[0]] for o in ops])
    vals = (C.c_int64 * n)(*[int(o[1]) if len(o) > 1 else 0 for o in ops])
    res = (C.c_int64 * n)()
    _check("swim_kat_collector", lib.swim_kat_collector(kinds, vals, n, res))
    return list(res)


# -- cell decoding (swim.h "Packed view cell") ----------------------------------------------
def cell_inc(c):
    return (np.asarray(c, dtype=np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)


def cell_status(c):
    return ((np.asarray(c, dtype=np.uint64) >> np.uint64(32)) & np.uint64(3)).astype(np.uint32)


def cell_flag(c, bit: int):
    return ((np.asarray(c, dtype=np.uint64) >> np.uint64(bit)) & np.uint64(1)).astype(bool)


def cell_in_table(c):
    return cell_flag(c, 34)


def cell_in_members(c):
    return cell_flag(c, 35)


def cell_has_timer(c):
    return cell_flag(c, 37)


def cell_deadline(c):
    return (np.asarray(c, dtype=np.uint64) >> np.uint64(39)).astype(np.uint32)


def debug_counters(lib, n: int = 16, reset: bool = False) -> list[int]:
    """swim_debug_counters: phase-timing sums of a profiling build (zeros otherwise)."""
    out = (C.c_uint64 * n)()
    _check("swim_debug_counters", lib.swim_debug_counters(out, n, 1 if reset else 0))
    return list(out)
