"""Consistency of the Java (Panama FFM) shim under java/ with the C ABI it binds (include/swim.h).

There is no JDK in this image, so the shim is not compiled here; these checks pin what a compile
would not catch anyway: every bound symbol exists in swim.h and in both libraries with the same
arity, the struct layouts list swim.h's fields in order, and the constants equal swim.h's.
"""
import ctypes
import os
import re

import pytest

import oracle
from swimgpu import load_library

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(REPO, "java", "src", "main", "java", "io", "scalecube", "cluster")
HEADER = open(os.path.join(REPO, "include", "swim.h")).read()
NATIVE = open(os.path.join(JAVA, "sim", "SwimNative.java")).read()


def _strip_comments(src):
    return re.sub(r"/\*.*?\*/", "", src, flags=re.S)


def c_struct_fields(name):
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), _strip_comments(HEADER), re.S).group(1)
    return re.findall(r"^\s*(?:u?int\d+_t|double)\s+(\w+)\s*(?:\[\d+\])?;", body, re.M)


def java_layout_fields(const):
    body = re.search(r"%s =\s*MemoryLayout\.structLayout\((.*?)\);" % const, NATIVE, re.S).group(1)
    return re.findall(r'withName\("(\w+)"\)', body)


def c_functions():
    out = {}
    for m in re.finditer(r"^(?:int32_t|size_t|int64_t)\s+(swim_\w+)\((.*?)\);", _strip_comments(HEADER), re.M | re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        out[m.group(1)] = len(args)
    return out


def java_handles():
    return {m.group(1): len([a for a in m.group(2).split(",") if a.strip()]) - 1
            for m in re.finditer(r'h\("(swim_\w+)",\s*([^)]*)\)', NATIVE)}


def test_config_layout_matches_header():
    assert java_layout_fields("CONFIG") == c_struct_fields("swim_config")


def test_event_layout_matches_header():
    assert java_layout_fields("EVENT") == c_struct_fields("swim_event")


def test_bound_symbols_exist_with_the_same_arity():
    decl = c_functions()
    handles = java_handles()
    assert len(handles) >= 25
    for name, nargs in handles.items():
        assert name in decl, name
        assert decl[name] == nargs, (name, decl[name], nargs)


@pytest.mark.parametrize("which", ["oracle", "gpu"])
def test_bound_symbols_are_exported(which):
    lib = oracle.lib() if which == "oracle" else load_library()
    for name in java_handles():
        assert isinstance(getattr(lib, name), ctypes._CFuncPtr), name


def test_constants_match_header():
    defines = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (SWIM_\w+) \(?(-?\d+)\)?", HEADER)}
    java = {m.group(1): int(m.group(2)) for m in re.finditer(r"public static final int (\w+) = (-?\d+);", NATIVE)}
    for jn, v in java.items():
        cn = {"ALL_MEMBERS": None}.get(jn, "SWIM_" + jn if not jn.startswith("SWIM_") else jn)
        if cn is None:
            continue
        assert defines.get(cn) == v, (jn, cn, defines.get(cn), v)


def test_views_implement_the_reference_interfaces():
    """Each view declares the reference interface and every one of its methods (the interface
    method lists of FailureDetector.java:12-25, GossipProtocol.java:12-29, MembershipProtocol.java:14-65)."""
    want = {
        ("fdetector", "SimFailureDetector", "FailureDetector"): ["start()", "stop()", "listen()"],
        ("gossip", "SimGossipProtocol", "GossipProtocol"): ["start()", "stop()", "spread(Message", "listen()"],
        ("membership", "SimMembershipProtocol", "MembershipProtocol"):
            ["start()", "stop()", "listen()", "members()", "otherMembers()", "member()", "member(String",
             "member(Address"],
    }
    for (pkg, cls, iface), methods in want.items():
        src = open(os.path.join(JAVA, pkg, cls + ".java")).read()
        assert f"class {cls} implements {iface}" in src
        for mth in methods:
            assert re.search(r"@Override\s+public [\w<>, ]+ " + re.escape(mth), src), (cls, mth)


# ---- behaviour: every SimNetworkEmulator method issues the same swim_* call sequence as the Python
# mirror (swimgpu/cluster.py NetworkEmulator), which the parity scenarios exercise against the
# reference semantics (NetworkEmulator.java:70-289).  The Java methods are written in a small subset
# (cluster.run lambda, for-each loops, call(...) statements, link bookkeeping) that is translated to
# Python here and run against a recorder, so the check reads the shim's actual method bodies.
EMU_SRC = open(os.path.join(JAVA, "sim", "SimNetworkEmulator.java")).read()

JAVA_TO_PY_NAMES = {"outboundSettings": "outbound_settings", "setDefaultOutboundSettings": "set_default_outbound_settings",
                    "blockAllOutbound": "block_all_outbound", "unblockAllOutbound": "unblock_all_outbound",
                    "blockOutbound": "block_outbound", "unblockOutbound": "unblock_outbound",
                    "inboundSettings": "inbound_settings", "setDefaultInboundSettings": "set_default_inbound_settings",
                    "blockAllInbound": "block_all_inbound", "unblockAllInbound": "unblock_all_inbound",
                    "blockInbound": "block_inbound", "unblockInbound": "unblock_inbound"}


def _java_methods(src):
    """name -> (params, python source of the body) for the public void methods of the emulator."""
    out = {}
    for m in re.finditer(r"public void (\w+)\(([^)]*)\) \{", src):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        body = src[m.end():i - 1]
        params = [p.split()[-1] for p in m.group(2).split(",") if p.strip()]
        lines, ind = [], 1
        for ln in body.splitlines():
            ln = ln.strip()
            if not ln or ln in ("cluster.run(() -> {", "});"):
                continue
            if ln == "}":
                ind -= 1
                continue
            fm = re.fullmatch(r"for \(int (\w+) : ([\w.()]+)\) \{", ln)
            if fm:
                lines.append("    " * ind + f"for {fm.group(1)} in {fm.group(2)}:")
                ind += 1
                continue
            ln = re.sub(r'call\(SwimNative\.\w+, ("\w+"), cluster\.engine\(\), ', r"call(\1, ", ln)
            ln = re.sub(r"(\w+) \? 1 : 0", r"(1 if \1 else 0)", ln)
            assert ln.endswith(";") and "(" in ln, ln
            lines.append("    " * ind + ln[:-1])
        out[m.group(1)] = (params, "\n".join(lines) or "    pass")
    return out


class _JavaCluster:
    """SimulatedCluster's link bookkeeping (TreeSet per member, removed by take*Links)."""

    def __init__(self):
        self.out, self.inn = {}, {}

    def checkLossPercent(self, pct):
        if not 0 <= pct <= 100:
            raise ValueError(pct)

    def noteOutLink(self, m, d):
        self.out.setdefault(m, set()).add(d)

    def noteInLink(self, m, s):
        self.inn.setdefault(m, set()).add(s)

    def takeOutLinks(self, m):
        return sorted(self.out.pop(m, ()))

    def takeInLinks(self, m):
        return sorted(self.inn.pop(m, ()))


class _Recorder:
    def __init__(self):
        self.calls = []

    def __getattr__(self, name):
        if not name.startswith("swim_"):
            raise AttributeError(name)
        return lambda h, *args: self.calls.append((name, *[int(a) for a in args])) or 0


def _python_mirror():
    from collections import defaultdict

    from swimgpu import abi, cluster
    rec = _Recorder()
    eng = abi.Engine.__new__(abi.Engine)
    eng.lib, eng._h = rec, None
    sc = cluster.SimulatedCluster.__new__(cluster.SimulatedCluster)
    sc.engine, sc._links, sc._inlinks = eng, defaultdict(set), defaultdict(set)
    return sc, rec


# a script of (member, method, args) exercising overrides followed by the clearing variants
EMU_SCRIPT = [
    (2, "outboundSettings", (5, 30, 200)), (2, "blockOutbound", ([7, 9],)), (2, "setDefaultOutboundSettings", (10, 50)),
    (2, "unblockOutbound", ([9],)), (2, "blockAllOutbound", ()), (2, "outboundSettings", (4, 0, 0)),
    (2, "unblockAllOutbound", ()), (2, "unblockAllOutbound", ()),
    (3, "inboundSettings", (1, True)), (3, "blockInbound", ([6, 8],)), (3, "setDefaultInboundSettings", (False,)),
    (3, "unblockInbound", ([8],)), (3, "blockAllInbound", ()), (3, "inboundSettings", (2, False)),
    (3, "unblockAllInbound", ()), (0, "blockOutbound", ([1],)), (0, "blockInbound", ([1],)),
    (0, "blockAllInbound", ()), (0, "blockAllOutbound", ()),
]


def test_network_emulator_shim_matches_python_mirror_call_for_call():
    methods = _java_methods(EMU_SRC)
    assert set(methods) == set(JAVA_TO_PY_NAMES), sorted(methods)
    jcalls = []
    jc = _JavaCluster()
    fns = {}
    for name, (params, body) in methods.items():
        src = f"def {name}(member, {', '.join(params)}):\n{body}\n" if params else f"def {name}(member):\n{body}\n"
        ns = {"cluster": jc, "call": lambda fn, *a: jcalls.append((fn, *[int(x) for x in a]))}
        exec(src, ns)
        fns[name] = ns[name]
    sc, rec = _python_mirror()
    from swimgpu import cluster
    for step, (m, name, args) in enumerate(EMU_SCRIPT):
        j0, p0 = len(jcalls), len(rec.calls)
        fns[name](m, *args)
        getattr(cluster.NetworkEmulator(sc, m), JAVA_TO_PY_NAMES[name])(*args)
        assert jcalls[j0:] == rec.calls[p0:], (step, name, jcalls[j0:], rec.calls[p0:])
    # the clearing variants removed every link override they had set
    assert ("swim_set_link_loss", 2, 5, -1) in jcalls and ("swim_set_link_inbound", 3, 1, -1) in jcalls
