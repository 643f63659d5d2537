"""Reference-timing discrete-event model of the protocol layer (SURVEY.md §7 build step 1b).

TEST INFRASTRUCTURE ONLY (like the rest of oracle/): a second restatement of the reference, this
one asynchronous.  Each virtual member runs the reference's control flow message by message on its
own timers, with the reference's timing: every member's FD / gossip / SYNC timers start at an
independent random phase (members of a real cluster start at different instants), messages take a
random localhost delay, and timeouts race with responses.  The lockstep engine (GPU and C++
oracle) fixes a canonical order on a 100-ms tick grid instead; this model is what
its detection-latency and convergence distributions are compared with (tests/test_ks_des.py, KS).

Restated from /root/reference/cluster/src/main/java/io/scalecube/cluster/:
  fdetector/FailureDetectorImpl.java   doPing :126-171, doPingReq :173-210, onPing :227-259,
                                       onPingReq :262-285, onTransitPingAck :291-315,
                                       selectPingMember :352-361, selectPingReqMembers :363-375,
                                       onMemberEvent :321-346
  gossip/GossipProtocolImpl.java       doSpreadGossip :141-184, onGossipReq :201-215,
                                       selectGossipMembers :322-343, selectGossipsToSend :311-320,
                                       sweep :350-368, onMemberEvent :238-261
  membership/MembershipProtocolImpl.java onFailureDetectorEvent :418-449, doSync :339-357,
                                       onSync :394-415, onSyncAck :363-391, updateMembership :569-664,
                                       onLeaving/onDead/onAlive :666-795, suspicion timers :797-834
  membership/MetadataStoreImpl.java    fetchMetadata :146-185 (one request/response round trip)
  transport: TransportImpl.requestResponse :214-238 (a response is matched by correlation id only,
  so the first relayed ack completes every pending relay request of that ping); a stopped
  member's transport refuses connections, so a send to it fails at the sender immediately.
Not modelled (quiet localhost cluster, one kill): loss / partitions, leave, joins, metadata
updates, namespaces, gossip segmentation (> 1000 intervals).
"""
from __future__ import annotations

import heapq
import random

ALIVE, SUSPECT, LEAVING, DEAD = 0, 1, 2, 3


def ceil_log2(n):  # ClusterMath.ceilLog2 (:133-135)
    return n.bit_length() if n > 0 else 0


def is_overrides(r1, r0):  # MembershipRecord.isOverrides (:67-88); records are (status, inc)
    if r0 is None:
        return r1[0] in (ALIVE, LEAVING)
    if r1 == r0:
        return False
    if r0[0] == DEAD:
        return False
    if r1[0] == DEAD:
        return True
    if r1[1] == r0[1]:
        return r1[0] == SUSPECT and r0[0] in (ALIVE, LEAVING)
    return r1[1] > r0[1]


class Member:
    def __init__(self, mid, n, rng):
        self.id = mid
        self.up = True
        others = [x for x in range(n) if x != mid]
        self.table = {x: (ALIVE, 0) for x in range(n)}
        self.members = set(range(n))
        self.alive_emitted = set(range(n)) - {mid}
        self.timers = {}  # subject -> suspicion timeout event id
        self.ping_members = others[:]
        rng.shuffle(self.ping_members)
        self.ping_idx = 0
        self.remote = others[:]
        rng.shuffle(self.remote)
        self.remote_idx = 0
        self.fd_period = 0
        self.g_period = 0
        self.g_counter = 0
        self.gossips = []  # [gossiper, seq, record(subject, status, inc), infection_period, infected]
        self.collectors = {}  # gossiper -> set of sequence ids


class Des:
    def __init__(self, n, seed, ping_interval=1000, ping_timeout=500, ping_req=3, gossip_interval=200,
                 fanout=3, repeat=3, sync_interval=30000, sync_timeout=3000, suspicion_mult=5,
                 metadata_timeout=3000, mean_delay_ms=0.5):
        self.n = n
        self.rng = random.Random(seed)
        self.cfg = dict(ping_interval=ping_interval, ping_timeout=ping_timeout, ping_req=ping_req,
                        gossip_interval=gossip_interval, fanout=fanout, repeat=repeat,
                        sync_interval=sync_interval, sync_timeout=sync_timeout, suspicion_mult=suspicion_mult,
                        metadata_timeout=metadata_timeout)
        self.mean_delay = mean_delay_ms
        self.now = 0.0
        self.q = []
        self.seq = 0
        self.cancelled = set()
        self.m = [Member(i, n, self.rng) for i in range(n)]
        self.pending = {}  # (member, cid) -> list of (on_ok, timeout event id)
        self.cid = 0
        self.log = []  # (time, viewer, kind, subject)
        self._firing = 0
        for mm in self.m:  # independent start instants (the members did not start together)
            self.after(self.rng.uniform(0, ping_interval), self.fd_tick, mm.id)
            self.after(self.rng.uniform(0, gossip_interval), self.gossip_tick, mm.id)
            self.after(self.rng.uniform(0, sync_interval), self.sync_tick, mm.id)

    # ---- event loop ----------------------------------------------------------------------------
    def after(self, dt, fn, *args):
        self.seq += 1
        heapq.heappush(self.q, (self.now + dt, self.seq, fn, args))
        return self.seq

    def cancel(self, eid):
        self.cancelled.add(eid)

    def run_until(self, t_end):
        while self.q and self.q[0][0] <= t_end:
            t, eid, fn, args = heapq.heappop(self.q)
            if eid in self.cancelled:
                self.cancelled.discard(eid)
                continue
            self.now = t
            self._firing = eid
            fn(*args)
        self.now = t_end

    def delay(self):
        return self.rng.expovariate(1.0 / self.mean_delay) if self.mean_delay > 0 else 0.0

    # ---- transport -----------------------------------------------------------------------------
    def send(self, src, dst, handler, *args):
        """Fire-and-forget send; False if dst's transport refuses the connection (stopped)."""
        if not self.m[dst].up:
            return False
        self.after(self.delay(), self._deliver, dst, handler, args)
        return True

    def _deliver(self, dst, handler, args):
        if self.m[dst].up:
            handler(dst, *args)

    def request(self, src, dst, cid, timeout, handler, args, on_ok, on_err):
        """requestResponse + timeout (TransportImpl.java:214-238): the response is whatever message
        with this correlation id reaches `src` first."""
        if not self.m[dst].up:
            on_err()
            return
        tid = self.after(timeout, self._timeout, src, cid, on_err)
        self.pending.setdefault((src, cid), []).append((on_ok, tid))
        self.after(self.delay(), self._deliver, dst, handler, args)

    def _timeout(self, src, cid, on_err):
        lst = self.pending.get((src, cid), [])
        for k, (_ok, tid) in enumerate(lst):  # drop exactly the request whose timer fired
            if tid == self._firing:
                lst.pop(k)
                break
        on_err()

    def respond(self, to, cid, payload):
        """A response travelling to `to`: completes every pending request of `to` with this cid."""
        def arrive(dst):
            for ok, tid in self.pending.pop((dst, cid), []):
                self.cancel(tid)
                ok(payload)
        self.send(None, to, arrive)

    # ---- failure detector (FailureDetectorImpl) --------------------------------------------------
    def fd_tick(self, v):
        mv = self.m[v]
        if not mv.up:
            return
        self.after(self.cfg["ping_interval"], self.fd_tick, v)
        mv.fd_period += 1
        if not mv.ping_members:
            return
        if mv.ping_idx >= len(mv.ping_members):  # selectPingMember :352-361
            mv.ping_idx = 0
            self.rng.shuffle(mv.ping_members)
        t = mv.ping_members[mv.ping_idx]
        mv.ping_idx += 1
        self.cid += 1
        cid = self.cid
        self.request(v, t, cid, self.cfg["ping_timeout"], self.on_ping, (v, cid),
                     lambda st, v=v, t=t: self.publish_fd(v, t, st),
                     lambda v=v, t=t, cid=cid: self.ping_failed(v, t, cid))

    def on_ping(self, me, frm, cid, issuer=None):
        self.respond(frm, cid, ALIVE)  # DEST_OK (no restarts here)

    def ping_failed(self, v, t, cid):
        mv = self.m[v]
        if not mv.up:
            return
        left = self.cfg["ping_interval"] - self.cfg["ping_timeout"]
        cands = [x for x in mv.ping_members if x != t]  # selectPingReqMembers :363-375
        self.rng.shuffle(cands)
        relays = cands[:self.cfg["ping_req"]]
        if left <= 0 or not relays:
            self.publish_fd(v, t, SUSPECT)
            return
        for r in relays:  # doPingReq :173-210, one request per relay, shared correlation id
            self.request(v, r, cid, left, self.on_ping_req, (v, t, cid),
                         lambda st, v=v, t=t: self.publish_fd(v, t, st),
                         lambda v=v, t=t: self.publish_fd(v, t, SUSPECT))

    def on_ping_req(self, relay, issuer, target, cid):
        # transit PING; a refused connection is only logged (:273-283)
        self.send(relay, target, self.on_transit_ping, relay, issuer, cid)

    def on_transit_ping(self, target, relay, issuer, cid):
        self.send(target, relay, self.on_transit_ack, issuer, cid)

    def on_transit_ack(self, relay, issuer, cid):
        self.respond(issuer, cid, ALIVE)

    def publish_fd(self, v, t, status):
        if not self.m[v].up:
            return
        if status == SUSPECT:
            self.log.append((self.now, v, "fd_suspect", t))
        self.on_fd_event(v, t, status)

    # ---- membership (MembershipProtocolImpl) -------------------------------------------------------
    def on_fd_event(self, v, t, status):  # :418-449
        mv = self.m[v]
        r0 = mv.table.get(t)
        if r0 is None or r0[0] == status:
            return
        if status == ALIVE:
            self.do_sync_to(v, t)
            return
        self.update(v, t, (status, r0[1]), "fd")

    def spread(self, v, subject, rec):  # spreadMembershipGossip -> createAndPutGossip
        mv = self.m[v]
        seq = mv.g_counter
        mv.g_counter += 1
        mv.gossips.append([v, seq, (subject, rec[0], rec[1]), mv.g_period, set()])
        mv.collectors.setdefault(v, set()).add(seq)

    def update(self, v, s, r1, reason):  # updateMembership :569-664
        mv = self.m[v]
        r0 = mv.table.get(s)
        leaving0 = r0 is not None and r0[0] == LEAVING
        if not leaving0 and not is_overrides(r1, r0):
            return
        if s == v:  # onSelfMemberDetected :686-708
            cur = max(r0[1], r1[1]) + 1
            mv.table[v] = (r0[0], cur)
            self.spread(v, v, (r0[0], cur))
            return
        if r1[0] == DEAD:  # onDeadMemberDetected :740-767
            tid = mv.timers.pop(s, None)
            if tid is not None:
                self.cancel(tid)
            if s not in mv.members:
                return
            mv.table.pop(s, None)
            mv.members.discard(s)
            mv.alive_emitted.discard(s)
            self.log.append((self.now, v, "removed", s))
            self.on_removed(v, s)
            return
        if r1[0] == SUSPECT:  # :621-628
            if not leaving0:
                if r0 is None or r0[0] != SUSPECT:
                    self.log.append((self.now, v, "suspect", s))
                mv.table[s] = r1
            if s not in mv.timers:  # computeIfAbsent
                ms = self.cfg["suspicion_mult"] * ceil_log2(len(mv.table)) * self.cfg["ping_interval"]
                mv.timers[s] = self.after(ms, self.suspicion_timeout, v, s)
            if reason not in ("gossip", "initial_sync"):
                self.spread(v, s, r1)
            return
        if r1[0] == ALIVE and (r0 is None or r0[1] < r1[1]):  # metadata round trip, then apply
            def ok(_p, v=v, s=s, r1=r1, reason=reason):
                self.apply_alive(v, s, r1, reason)
            self.cid += 1
            self.request(v, s, ("meta", self.cid), self.cfg["metadata_timeout"], self.on_meta_req,
                         (v, ("meta", self.cid)), ok, lambda: None)

    def on_meta_req(self, me, frm, cid):
        self.respond(frm, cid, None)

    def apply_alive(self, v, s, r1, reason):  # :648-656 + onAliveMemberDetected :769-795
        mv = self.m[v]
        if not mv.up:
            return
        tid = mv.timers.pop(s, None)
        if tid is not None:
            self.cancel(tid)
        if reason not in ("gossip", "initial_sync"):
            self.spread(v, s, r1)
        mv.table[s] = r1
        mv.members.add(s)

    def suspicion_timeout(self, v, s):  # :825-834
        mv = self.m[v]
        mv.timers.pop(s, None)
        if not mv.up:
            return
        r0 = mv.table.get(s)
        if r0 is not None:
            self.update(v, s, (DEAD, r0[1]), "timeout")

    def on_removed(self, v, s):  # FD / gossip onMemberEvent REMOVED
        mv = self.m[v]
        if s in mv.ping_members:
            mv.ping_members.remove(s)
        if s in mv.remote:
            mv.remote.remove(s)
        mv.collectors.pop(s, None)

    def sync_tick(self, v):  # doSync :339-357
        mv = self.m[v]
        if not mv.up:
            return
        self.after(self.cfg["sync_interval"], self.sync_tick, v)
        others = sorted(mv.members - {v})
        if others:
            self.do_sync_to(v, self.rng.choice(others))

    def do_sync_to(self, v, t):
        self.cid += 1
        rows = dict(self.m[v].table)
        self.request(v, t, ("sync", self.cid), self.cfg["sync_timeout"], self.on_sync, (v, ("sync", self.cid), rows),
                     lambda ack_rows, v=v: self.sync_merge(v, ack_rows), lambda: None)

    def on_sync(self, me, frm, cid, rows):  # :394-415
        self.sync_merge(me, rows)
        self.respond(frm, cid, dict(self.m[me].table))

    def sync_merge(self, v, rows):  # syncMembership :491-509
        if not self.m[v].up:
            return
        for s in sorted(rows):
            self.update(v, s, rows[s], "sync")

    # ---- gossip (GossipProtocolImpl) ----------------------------------------------------------------
    def gossip_tick(self, v):  # doSpreadGossip :141-184
        mv = self.m[v]
        if not mv.up:
            return
        self.after(self.cfg["gossip_interval"], self.gossip_tick, v)
        period = mv.g_period
        mv.g_period += 1
        if not mv.gossips:
            return
        f = self.cfg["fanout"]
        if len(mv.remote) < f:
            targets = mv.remote[:]
        else:
            if mv.remote_idx + f > len(mv.remote):
                self.rng.shuffle(mv.remote)
                mv.remote_idx = 0
            targets = mv.remote[mv.remote_idx:mv.remote_idx + f]
            mv.remote_idx += f
        spread = self.cfg["repeat"] * ceil_log2(len(mv.remote) + 1)
        sweep = 2 * (spread + 1)
        for t in targets:
            for g in mv.gossips:
                if g[3] + spread >= period and t not in g[4]:
                    self.send(v, t, self.on_gossip, v, g[0], g[1], g[2])
        mv.gossips = [g for g in mv.gossips if not period > g[3] + sweep]

    def on_gossip(self, r, frm, gossiper, seq, rec):  # onGossipReq :201-215
        mr = self.m[r]
        col = mr.collectors.setdefault(gossiper, set())
        if seq in col:
            return
        col.add(seq)
        mr.gossips.append([gossiper, seq, rec, mr.g_period, {frm}])
        self.update(r, rec[0], (rec[1], rec[2]), "gossip")

    # ---- scenario ----------------------------------------------------------------------------------
    def kill(self, v):
        self.m[v].up = False


def kill_run(n, seed, victim, t_kill_ms, t_end_ms, **cfg):
    """One run: converged cluster, `victim` stopped at t_kill; returns the log."""
    d = Des(n, seed, **cfg)
    d.run_until(t_kill_ms)
    d.kill(victim)
    d.run_until(t_end_ms)
    return d.log


def run_stats(log, victim, viewer, t_kill, n_live):
    """Per-run statistics, ms after the kill (None where the run did not get there):
    detect   first FailureDetector SUSPECT of the victim published by any member,
    suspect  `viewer`'s table first shows the victim SUSPECT (FD or gossip),
    removed  `viewer` emits REMOVED for the victim,
    converge the last live member emits REMOVED (all live views agree)."""
    fd = [t for t, v, k, s in log if k == "fd_suspect" and s == victim and t >= t_kill]
    sus = [t for t, v, k, s in log if k == "suspect" and s == victim and v == viewer and t >= t_kill]
    rem_v = [t for t, v, k, s in log if k == "removed" and s == victim and v == viewer]
    rem = sorted(t for t, v, k, s in log if k == "removed" and s == victim)
    f = lambda xs: (min(xs) - t_kill) if xs else None  # noqa: E731
    return {"detect": f(fd), "suspect": f(sus), "removed": f(rem_v),
            "converge": (rem[-1] - t_kill) if len(rem) == n_live else None}


def des_sample(n, seed, horizon_ms, **cfg):
    """One DES run with the victim, the observed viewer and the kill instant drawn from `seed`."""
    rng = random.Random(seed * 7919 + 17)
    victim = rng.randrange(n)
    viewer = rng.choice([x for x in range(n) if x != victim])
    t_kill = 10000.0 + rng.uniform(0, cfg.get("ping_interval", 1000))
    log = kill_run(n, seed, victim, t_kill, t_kill + horizon_ms, **cfg)
    return run_stats(log, victim, viewer, t_kill, n - 1)


if __name__ == "__main__":
    import time
    t0 = time.time()
    print(des_sample(64, 1, 60000.0), f"{time.time() - t0:.2f}s")
