"""Transcribe the reference's known-answer tests into tests/golden/reference_kats.json.

Reads (as text) the two JUnit files of the reference that pin the merge and dedupe arithmetic:
  cluster/src/test/java/io/scalecube/cluster/membership/MembershipRecordTest.java
  cluster/src/test/java/io/scalecube/cluster/gossip/SequenceIdCollectorTest.java
and turns every assertion into a data row (inputs, expected output, source line).  Run here, where
/root/reference exists; the tests only load the committed JSON.

    python tests/golden/transcribe_reference_kats.py [/root/reference]
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
MRT = "cluster/src/test/java/io/scalecube/cluster/membership/MembershipRecordTest.java"
SICT = "cluster/src/test/java/io/scalecube/cluster/gossip/SequenceIdCollectorTest.java"
STATUS = {"ALIVE": 0, "SUSPECT": 1, "LEAVING": 2, "DEAD": 3}


def membership_record_test(path):
    lines = open(path).read().splitlines()
    recs = {}
    defn = re.compile(r"MembershipRecord (\w+) = (?:new MembershipRecord\(member, (\w+), (\d+)\)|null)")
    for ln in lines:
        m = defn.search(ln)
        if m:
            recs[m.group(1)] = None if m.group(2) is None else [STATUS[m.group(2)], int(m.group(3))]
    rows, test = [], None
    asrt = re.compile(r"assert(True|False)\((\w+)\.isOverrides\((\w+)\)\)")
    for no, ln in enumerate(lines, 1):
        t = re.search(r"public void (\w+)\(", ln)
        if t:
            test = t.group(1)
        m = asrt.search(ln)
        if m:
            rows.append({"test": test, "line": no, "r1": recs[m.group(2)], "r0": recs[m.group(3)],
                         "overrides": m.group(1) == "True"})
    return rows


def sequence_id_collector_test(path):
    """A small interpreter for the test bodies: add / contains / size / clear, for-loops of add."""
    lines = open(path).read().splitlines()
    tests, cur, loop = {}, None, None
    for no, ln in enumerate(lines, 1):
        s = ln.strip()
        t = re.search(r"public void (\w+)\(", s)
        if t:
            cur = tests.setdefault(t.group(1), {"line": no, "ops": []})
            continue
        if cur is None:
            continue
        m = re.match(r"for \(int i = (\d+); i < (\d+); i\+\+\) \{", s)
        if m:
            loop = (int(m.group(1)), int(m.group(2)))
            continue
        if s == "}" and loop:
            loop = None
            continue
        m = re.match(r"assert(True|False)\(sequenceIdCollector\.(add|contains)\((\w+)\)\);", s)
        if m:
            vals = range(*loop) if (loop and m.group(3) == "i") else [int(m.group(3))]
            for v in vals:
                cur["ops"].append({"op": m.group(2), "value": v, "expect": 1 if m.group(1) == "True" else 0,
                                   "line": no})
            continue
        m = re.match(r"assertEquals\((\d+), sequenceIdCollector\.size\(\)\);", s)
        if m:
            cur["ops"].append({"op": "size", "expect": int(m.group(1)), "line": no})
            continue
        m = re.match(r"sequenceIdCollector\.(add|clear)\((\w*)\);", s)
        if m:  # un-asserted call: its result is not pinned
            op = {"op": m.group(1), "line": no, "expect": None}
            if m.group(2):
                op["value"] = int(m.group(2))
            cur["ops"].append(op)
    return {k: v for k, v in tests.items() if v["ops"]}


def main():
    doc = {
        "source": "transcribed by tests/golden/transcribe_reference_kats.py from the reference's JUnit tests",
        "MembershipRecordTest": {"file": MRT, "cases": membership_record_test(os.path.join(REF, MRT))},
        "SequenceIdCollectorTest": {"file": SICT, "tests": sequence_id_collector_test(os.path.join(REF, SICT))},
    }
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    n1 = len(doc["MembershipRecordTest"]["cases"])
    n2 = sum(len(t["ops"]) for t in doc["SequenceIdCollectorTest"]["tests"].values())
    print(f"wrote {out}: {n1} isOverrides assertions, {n2} collector ops")


if __name__ == "__main__":
    main()
