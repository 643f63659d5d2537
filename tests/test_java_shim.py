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
