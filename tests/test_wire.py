"""Wire format of the protocol messages (swimgpu/wire.py): JDK object serialization
as JdkMessageCodec produces it for the Externalizable records.

Parity **unpinned**: no JVM exists in this image to produce reference bytes, so these tests pin the
Java Object Serialization Stream Protocol constants and layout rules the codec restates (hand-assembled
expected streams), java.lang.String.hashCode / java.util.HashMap iteration order on the header map,
the round trip of every message type, and the bridge from engine state (a SYNC's SyncData from a
view row of the CPU oracle).
"""
import struct

import numpy as np
import pytest

from swimgpu import abi, wire


def utf(s):  # DataOutput.writeUTF for ASCII
    return struct.pack(">H", len(s)) + s.encode()


def desc(name, suid, flags):  # TC_CLASSDESC, name, suid, flags, no fields, no annotation
    return bytes([wire.TC_CLASSDESC]) + utf(name) + struct.pack(">qBh", suid, flags, 0) + bytes([wire.TC_ENDBLOCKDATA])


def test_java_string_hash_and_hashmap_order():
    # String.hashCode: s[0]*31^(n-1) + ... + s[n-1] as a signed int (Java SE API examples)
    assert wire.java_string_hash("") == 0
    assert wire.java_string_hash("q") == 113
    assert wire.java_string_hash("hello") == 99162322
    assert wire.java_string_hash("cid") == 98494
    assert wire.java_string_hash("sender") == -905962955
    # a 16-bucket HashMap: index (h ^ h >>> 16) & 15 -> q: 1, sender: 5, cid: 15
    for k, b in (("q", 1), ("sender", 5), ("cid", 15)):
        h = wire.java_string_hash(k) & 0xFFFFFFFF
        assert (h ^ (h >> 16)) & 15 == b
    got = wire.java_hashmap_order([("cid", "7"), ("sender", "h:1"), ("q", "sc/membership/sync")])
    assert [k for k, _ in got] == ["q", "sender", "cid"]


def test_modified_utf8():
    out = wire.ObjectOutput()
    out.write_utf("a\x00é€\U0001F600")
    b = out.getvalue()[4:]
    # NUL as C0 80; U+00E9 two bytes; U+20AC three; U+1F600 as two 3-byte surrogates
    body = b"a" + b"\xc0\x80" + b"\xc3\xa9" + b"\xe2\x82\xac" + b"\xed\xa0\xbd" + b"\xed\xb8\x80"
    assert b == bytes([wire.TC_BLOCKDATA, 2 + len(body)]) + struct.pack(">H", len(body)) + body
    assert wire.ObjectInput(wire.ObjectOutput().getvalue() + b).read_utf() == "a\x00é€\U0001F600"


def test_get_metadata_request_stream_layout():
    """A GET_METADATA request, byte for byte from the stream protocol: header block, the request
    object (descriptor, handle 0x7E0000 / object 0x7E0001), the Member inside it (descriptor 0x7E0002,
    object 0x7E0003) in its own block, end markers."""
    m = wire.Member("ab12", "10.0.0.1:4801", "ns")
    msg = wire.Message(((wire.HEADER_QUALIFIER, wire.GET_METADATA_REQ),), wire.GetMetadataRequest(m))
    hdr = struct.pack(">i", 1) + utf("q") + utf("sc/metadata/req")
    member_body = utf("ab12") + b"\x00" + utf("10.0.0.1:4801") + utf("ns")
    want = (struct.pack(">HH", 0xACED, 5) + bytes([wire.TC_BLOCKDATA, len(hdr)]) + hdr
            + bytes([wire.TC_OBJECT]) + desc("io.scalecube.cluster.metadata.GetMetadataRequest", 1, 0x0C) + bytes([wire.TC_NULL])
            + bytes([wire.TC_OBJECT]) + desc("io.scalecube.cluster.Member", 1, 0x0C) + bytes([wire.TC_NULL])
            + bytes([wire.TC_BLOCKDATA, len(member_body)]) + member_body + bytes([wire.TC_ENDBLOCKDATA])
            + bytes([wire.TC_ENDBLOCKDATA]))
    assert wire.serialize(msg) == want
    assert wire.deserialize(want) == msg


def test_sync_data_back_references():
    """Repeated class descriptors and repeated enum constants are TC_REFERENCEs.  Handles follow
    ObjectOutputStream's order (a descriptor is assigned before the object it describes): SyncData
    descriptor 0x7E0000, SyncData 0x7E0001, MembershipRecord descriptor 0x7E0002, record 0x7E0003,
    Member descriptor 0x7E0004, Member 0x7E0005, MemberStatus descriptor 0x7E0006, java.lang.Enum
    descriptor 0x7E0007, ALIVE 0x7E0008, its name 0x7E0009; the second record refers back to
    0x7E0002, 0x7E0004 and 0x7E0008."""
    recs = tuple(wire.MembershipRecord(wire.Member(f"m{i}", f"h:{i}"), 0, i) for i in range(2))
    b = wire.serialize(wire.Message((), wire.SyncData(recs)))
    ref = lambda h: bytes([wire.TC_REFERENCE]) + struct.pack(">i", h)
    i2 = b.index(b"m1") - 2  # the second Member's block data starts before its id's UTF length
    second = b[:i2]
    assert second.count(desc("io.scalecube.cluster.membership.MembershipRecord", 1, 0x0C)) == 1
    assert ref(0x7E0002) in b and ref(0x7E0004) in b and ref(0x7E0008) in b
    enum_chain = (bytes([wire.TC_ENUM]) + desc("io.scalecube.cluster.membership.MemberStatus", 0, 0x12)
                  + desc("java.lang.Enum", 0, 0x12) + bytes([wire.TC_NULL]) + bytes([wire.TC_STRING]) + utf("ALIVE"))
    assert b.count(enum_chain) == 1
    assert wire.deserialize(b).data == wire.SyncData(recs)


def test_block_data_is_chunked_at_1024_bytes():
    meta = bytes(range(256)) * 12  # 3,072 bytes of metadata
    msg = wire.Message((), wire.GetMetadataResponse(wire.Member("x", "h:1"), meta))
    b = wire.serialize(msg)
    # after the Member object: writeInt(3072) + 3,072 bytes = 3,076 bytes of block data, cut into
    # blocks of exactly 1,024 bytes (three TC_BLOCKDATALONG) and a 4-byte TC_BLOCKDATA
    longs = [i for i in range(len(b) - 5) if b[i] == wire.TC_BLOCKDATALONG and b[i + 1:i + 5] == struct.pack(">i", 1024)]
    assert len(longs) == 3
    assert wire.deserialize(b) == msg


@pytest.mark.parametrize("kind", ["ping", "ping_ack_gone", "sync", "gossip", "metadata_resp", "null_data"])
def test_round_trip(kind):
    a, b, c = (wire.Member(f"{i:08x}", f"localhost:{4800 + i}", "ns/x", alias="alias" if i == 1 else None) for i in range(3))
    data = {
        "ping": wire.PingData(a, b),
        "ping_ack_gone": wire.PingData(a, b, c, gone=True),
        "sync": wire.SyncData(tuple(wire.MembershipRecord(m, s, 7 + s) for m, s in ((a, 0), (b, 1), (c, 3)))),
        "gossip": wire.GossipRequest((wire.Gossip(a.id, wire.Message((("q", wire.MEMBERSHIP_GOSSIP),),
                                                                     wire.MembershipRecord(b, 2, 3)), 41),
                                      wire.Gossip(c.id, wire.Message((("q", wire.MEMBERSHIP_GOSSIP),),
                                                                     wire.MembershipRecord(a, 1, 0)), 42)), a.id),
        "metadata_resp": wire.GetMetadataResponse(c, b"\x01\x02\x03"),
        "null_data": None,
    }[kind]
    msg = wire.Message((("q", "sc/x"), ("cid", "1234"), ("sender", "localhost:4800")), data)
    back = wire.deserialize(wire.serialize(msg))
    assert back.data == msg.data
    assert dict(back.headers) == dict(msg.headers)


def test_sync_message_from_engine_view():
    """The SYNC a simulated member would put on the wire: its table from the engine (CPU oracle, the
    same ABI as libswimgpu), after one member was killed and suspected."""
    import oracle
    lib = oracle.lib()
    e = abi.Engine(lib, abi.default_config(lib), 8, 8, seed=3)
    e.step(2)
    e.kill(5)
    e.step(4)
    d = wire.Directory.local(8)
    msg = wire.sync_message(e, 0, d, cid="c1")
    back = wire.deserialize(wire.serialize(msg))
    row = e.read_view(0)
    recs = back.data.membership
    intab = np.flatnonzero((row >> 34) & 1)
    assert [r.member.id for r in recs] == [d.ids[s] for s in intab]
    for r, s in zip(recs, intab):
        assert r.status == (int(row[s]) >> 32) & 3 and r.incarnation == int(row[s]) & 0xFFFFFFFF
        assert r.member.address == f"localhost:{4800 + s}"
    assert back.header("q") == wire.SYNC and back.header("cid") == "c1"


def test_relayed_message_keeps_the_deserialised_map_capacity():
    """Message.readExternal builds `new HashMap<>(headersSize)` (Message.java:218-230), so a message a
    JVM deserialised and sends on (GossipProtocolImpl re-sends the Gossip objects it received) iterates
    its headers in buckets of tableSizeFor(n) plus resizes, not in the Builder's 16 buckets
    (Message.java:234).  Two headers whose bucket indices differ in bits 2-3 come out in opposite
    orders; a deserialised message re-serialises in the read map's order."""
    def bucket(k, cap):
        h = wire.java_string_hash(k) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)
    names = [f"h{i}" for i in range(200)]
    a, b = next((x, y) for x in names for y in names
                if bucket(x, 16) > bucket(y, 16) and bucket(x, 4) < bucket(y, 4))
    # new HashMap<>(2): a 2-bucket table, resized to 4 by the second put
    assert [k for k, _ in wire.java_hashmap_order([(a, "1"), (b, "2")], 2)] == [a, b]
    assert [k for k, _ in wire.java_hashmap_order([(a, "1"), (b, "2")])] == [b, a]
    built = wire.Message(((a, "1"), (b, "2")), None)
    raw = wire.serialize(built)
    assert raw.index(utf(b)) < raw.index(utf(a))
    back = wire.deserialize(raw)
    assert dict(back.headers) == dict(built.headers) and back.map_capacity == 2
    again = wire.serialize(back)
    assert again.index(utf(a)) < again.index(utf(b))
    # one header, and three (tableSizeFor(3) = 4, resized to 8 at the third put): sizes past a resize
    assert [k for k, _ in wire.java_hashmap_order([(a, "1")], 1)] == [a]
    three = [(f"k{i}", str(i)) for i in range(3)]
    got = [k for k, _ in wire.java_hashmap_order(three, 3)]
    assert got == sorted((k for k, _ in three), key=lambda k: (bucket(k, 8), int(k[1:])))


def test_ingest_external_sync_ack():
    """swim_ingest_sync (onSyncAck, MembershipProtocolImpl.java:363-391) fed from the wire: a SYNC_ACK
    a JVM node would send, decoded and mapped onto the engine's slots (unknown ids dropped), merged into
    a viewer of the CPU oracle (the GPU path is compared with it in the external_sync_16 scenario).
    Parity with a JVM unpinned (no JVM here)."""
    import oracle
    lib = oracle.lib()
    e = abi.Engine(lib, abi.default_config(lib), 8, 8, seed=5)
    e.step(2)
    d = wire.Directory.local(8)
    recs = (wire.MembershipRecord(d.member(4), abi.SUSPECT, 0), wire.MembershipRecord(d.member(2), abi.SUSPECT, 0),
            wire.MembershipRecord(d.member(6), abi.ALIVE, 0),  # equal incarnation: no change
            wire.MembershipRecord(wire.Member("beef", "other:1"), abi.ALIVE, 3))
    msg = wire.Message(((wire.HEADER_QUALIFIER, wire.SYNC_ACK),), wire.SyncData(recs))
    got = wire.engine_records(wire.deserialize(wire.serialize(msg)), d)
    assert got == [(4, abi.SUSPECT, 0), (2, abi.SUSPECT, 0), (6, abi.ALIVE, 0)]
    before = e.stats()
    e.drain_events()
    e.ingest_sync(2, got)
    row = e.read_view(2).astype(np.int64)
    st = lambda s: int(row[s] >> 32) & 3
    inc = lambda s: int(row[s] & 0xFFFFFFFF)
    assert (st(4), inc(4)) == (abi.SUSPECT, 0)   # suspected, suspicion timer scheduled
    assert (st(2), inc(2)) == (abi.ALIVE, 1)     # a SUSPECT record of the viewer itself: refuted
    assert (st(6), inc(6)) == (abi.ALIVE, 0)
    g = e.read_gossips(2)
    assert sorted(int(x) for x in g["subject"]) == [2, 4]  # the refutation and the suspicion spread
    after = e.stats()
    assert after["sync_acks"] == before["sync_acks"] + 1
    assert after["sync_records"] == before["sync_records"] + 3
    # refused: a stopped viewer, a DEAD record (a SyncData never holds one), an out-of-range member
    e.kill(7)
    with pytest.raises(RuntimeError):
        e.ingest_sync(7, [(1, abi.ALIVE, 0)])
    with pytest.raises(RuntimeError):
        e.ingest_sync(1, [(3, abi.DEAD, 0)])
    with pytest.raises(RuntimeError):
        e.ingest_sync(1, [(8, abi.ALIVE, 0)])
    e.ingest_sync(1, [])  # an empty table is a no-op apart from the counters
    e.step(30)
    assert e.stats()["capacity_errors"] == 0
