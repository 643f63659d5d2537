"""Full-state comparison of two engines (GPU engine vs CPU oracle) through the swim.h readback ABI."""
from __future__ import annotations

import numpy as np

from swimgpu import abi

MEMBER_FIELDS = ("up", "joined", "leave_pending", "join_pending", "remote_idx", "fd_period", "ping_cursor",
                 "ping_len", "remote_len", "gossip_len", "gossip_period", "gossip_counter", "table_size",
                 "members_size", "fd_start", "gossip_start", "sync_start", "sync_on", "ack_target", "ack_due",
                 "relay_target", "relay_pending", "relay_due", "leave_gossiper", "leave_seq", "pending_acks")

STAT_FIELDS = ("pings", "ping_reqs", "fd_events", "gossips_created", "gossip_messages", "gossip_accepted",
               "syncs", "sync_acks", "sync_records", "fetches", "fetch_ok", "timers_fired", "events") + tuple(
                   f"orig_{r}" for r in abi.ORIG_REASONS)


def state_digest(e: abi.Engine, members=None, collectors=True) -> dict:
    n = e.capacity
    members = range(n) if members is None else members
    d = {"rows": {}, "members": {}, "ping": {}, "remote": {}, "gossips": {}, "coll": {}}
    for m in members:
        d["rows"][m] = e.read_view(m)
        ms = e.read_member(m)
        d["members"][m] = {k: ms[k] for k in MEMBER_FIELDS}
        d["ping"][m] = e.read_ping_list(m)
        d["remote"][m] = e.read_remote_list(m)
        g = e.read_gossips(m)
        d["gossips"][m] = g
        if collectors:
            gossipers = set(int(x) for x in g["gossiper"]) | {m}
            d["coll"][m] = {x: e.read_collector(m, x) for x in sorted(gossipers)}
    return d


def diff_states(a: dict, b: dict, limit: int = 12) -> list[str]:
    out = []
    for m in a["rows"]:
        ra, rb = a["rows"][m], b["rows"][m]
        if not np.array_equal(ra, rb):
            idx = np.nonzero(ra != rb)[0]
            out.append(f"row {m}: {len(idx)} cells differ, first {[(int(i), hex(int(ra[i])), hex(int(rb[i]))) for i in idx[:4]]}")
        for k in MEMBER_FIELDS:
            if a["members"][m][k] != b["members"][m][k]:
                out.append(f"member {m}.{k}: {a['members'][m][k]} != {b['members'][m][k]}")
        for key in ("ping", "remote"):
            if not np.array_equal(a[key][m], b[key][m]):
                out.append(f"{key} list {m}: {a[key][m][:16]} != {b[key][m][:16]}")
        if not np.array_equal(a["gossips"][m], b["gossips"][m]):
            out.append(f"gossips {m}: {a['gossips'][m][:4]} != {b['gossips'][m][:4]}")
        if a["coll"].get(m) != b["coll"].get(m):
            out.append(f"collectors {m}: {a['coll'].get(m)} != {b['coll'].get(m)}")
        if len(out) >= limit:
            break
    return out


def diff_events(ea: np.ndarray, eb: np.ndarray) -> list[str]:
    fields = ("tick", "viewer", "subject", "type", "phase", "minor")
    if len(ea) != len(eb):
        return [f"event count {len(ea)} != {len(eb)}"]
    for f in fields:
        if not np.array_equal(ea[f], eb[f]):
            i = int(np.nonzero(ea[f] != eb[f])[0][0])
            return [f"event {i} field {f}: {ea[i]} != {eb[i]}"]
    return []


def diff_stats(sa: dict, sb: dict) -> list[str]:
    return [f"stat {k}: {sa[k]} != {sb[k]}" for k in STAT_FIELDS if sa[k] != sb[k]]
