"""Wire format of the cluster protocol's messages: the bytes a JVM node running
scalecube-cluster puts on the transport for a Message, so that simulated members' state can be
shipped to (and read from) real nodes.

The transport's default codec (`MessageCodec.INSTANCE` falls back to `JdkMessageCodec` when no
Jackson codec is on the classpath, transport-api/.../MessageCodec.java:10-11) is JDK object
serialization: `JdkMessageCodec.serialize` (:20-25) opens an ObjectOutputStream and calls
`Message.writeExternal` directly (Message.java:206-215: header count, (name, value) UTF pairs in
the header map's iteration order, then `writeObject(data)`).  The data classes are Externalizable
with serialVersionUID 1 (so the stream is fully determined by their writeExternal bodies):

  Member            writeUTF id, writeBoolean alias != null, [writeUTF alias], writeUTF address,
                    writeUTF namespace                               (cluster-api Member.java:104-117)
  MembershipRecord  writeObject member, writeObject status (enum), writeInt incarnation
                                                                     (MembershipRecord.java:110-117)
  SyncData          writeInt size, writeObject record...             (SyncData.java:37-44)
  Gossip            writeUTF gossiperId, writeObject message, writeLong sequenceId (Gossip.java:65-72)
  GossipRequest     writeInt size, writeObject gossip..., writeUTF from (GossipRequest.java:43-51)
  PingData          writeObject from, to, originalIssuer, ackType (enum) (PingData.java:87-96)
  GetMetadataRequest   writeObject member                           (GetMetadataRequest.java:30-33)
  GetMetadataResponse  writeObject member, writeInt len, write bytes (GetMetadataResponse.java:41-48)

This module restates the subset of the Java Object Serialization Stream Protocol (version 2) those
classes exercise: stream header, block-data mode (1,024-byte blocks, TC_BLOCKDATA /
TC_BLOCKDATALONG), TC_OBJECT of Externalizable classes (class descriptor flags SC_EXTERNALIZABLE |
SC_BLOCK_DATA, no fields, TC_ENDBLOCKDATA after writeExternal), TC_ENUM (descriptor chain enum ->
java.lang.Enum, serialVersionUID 0, flags SC_SERIALIZABLE | SC_ENUM, the constant's name as
TC_STRING), TC_NULL, TC_STRING, and back-references (TC_REFERENCE to handles from 0x7E0000, assigned
in ObjectOutputStream's order: a class descriptor before its body, an object after its descriptor).
Java's HashMap iteration order of the header map (String.hashCode, spread, power-of-two table) is
restated too.  Address is `io.scalecube.net.Address` of scalecube-commons (not in the reference tree);
its toString is host:port.

Parity: **unpinned** — there is no JVM in this image to produce reference bytes; the tests pin the
protocol constants, the structure and the round trip (tests/test_wire.py).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any

# java.io.ObjectStreamConstants
STREAM_MAGIC, STREAM_VERSION = 0xACED, 5
TC_NULL, TC_REFERENCE, TC_CLASSDESC, TC_OBJECT, TC_STRING = 0x70, 0x71, 0x72, 0x73, 0x74
TC_BLOCKDATA, TC_ENDBLOCKDATA, TC_BLOCKDATALONG, TC_LONGSTRING, TC_ENUM = 0x77, 0x78, 0x7A, 0x7C, 0x7E
SC_SERIALIZABLE, SC_EXTERNALIZABLE, SC_BLOCK_DATA, SC_ENUM = 0x02, 0x04, 0x08, 0x10
BASE_HANDLE = 0x7E0000
MAX_BLOCK = 1024  # ObjectOutputStream.BlockDataOutputStream.MAX_BLOCK_SIZE

# qualifiers (FailureDetectorImpl.java:35-37, GossipProtocolImpl.java:38, MembershipProtocolImpl.java:68-70,
# MetadataStoreImpl.java:28-29) and header names (Message.java:27-39)
PING, PING_REQ, PING_ACK = "sc/fdetector/ping", "sc/fdetector/pingReq", "sc/fdetector/pingAck"
GOSSIP_REQ = "sc/gossip/req"
SYNC, SYNC_ACK, MEMBERSHIP_GOSSIP = "sc/membership/sync", "sc/membership/syncAck", "sc/membership/gossip"
GET_METADATA_REQ, GET_METADATA_RESP = "sc/metadata/req", "sc/metadata/resp"
HEADER_QUALIFIER, HEADER_CORRELATION_ID, HEADER_SENDER = "q", "cid", "sender"

MEMBER_STATUS = ("ALIVE", "SUSPECT", "LEAVING", "DEAD")  # MemberStatus.java (swim.h SWIM_* order)
ACK_TYPE = ("DEST_OK", "DEST_GONE")                      # PingData.AckType


# ------------------------------------------------------------------------------- data classes
@dataclass(frozen=True)
class Member:
    id: str
    address: str
    namespace: str = "default"
    alias: str | None = None
    JAVA = "io.scalecube.cluster.Member"

    def write_external(self, out: "ObjectOutput") -> None:
        out.write_utf(self.id)
        out.write_boolean(self.alias is not None)
        if self.alias is not None:
            out.write_utf(self.alias)
        out.write_utf(self.address)
        out.write_utf(self.namespace)

    @classmethod
    def read_external(cls, inp: "ObjectInput") -> "Member":
        mid = inp.read_utf()
        alias = inp.read_utf() if inp.read_boolean() else None
        addr = inp.read_utf()
        return cls(mid, addr, inp.read_utf(), alias)


@dataclass(frozen=True)
class JavaEnum:
    cls: str
    name: str


def member_status(s: int) -> JavaEnum:
    return JavaEnum("io.scalecube.cluster.membership.MemberStatus", MEMBER_STATUS[s])


def ack_type(gone: bool) -> JavaEnum:
    return JavaEnum("io.scalecube.cluster.fdetector.PingData$AckType", ACK_TYPE[1 if gone else 0])


@dataclass(frozen=True)
class MembershipRecord:
    member: Member
    status: int  # SWIM_ALIVE .. SWIM_DEAD
    incarnation: int
    JAVA = "io.scalecube.cluster.membership.MembershipRecord"

    def write_external(self, out):
        out.write_object(self.member)
        out.write_object(member_status(self.status))
        out.write_int(self.incarnation)

    @classmethod
    def read_external(cls, inp):
        m = inp.read_object()
        st = inp.read_object()
        return cls(m, MEMBER_STATUS.index(st.name), inp.read_int())


@dataclass(frozen=True)
class SyncData:
    membership: tuple
    JAVA = "io.scalecube.cluster.membership.SyncData"

    def write_external(self, out):
        out.write_int(len(self.membership))
        for r in self.membership:
            out.write_object(r)

    @classmethod
    def read_external(cls, inp):
        return cls(tuple(inp.read_object() for _ in range(inp.read_int())))


@dataclass(frozen=True)
class Message:
    headers: tuple  # ((name, value), ...) in insertion order; serialised in HashMap order
    data: Any = None
    # the header map's construction: None = Message.Builder's `new HashMap<>()`; n = readExternal's
    # `new HashMap<>(n)` (a message a JVM deserialised and re-sends, e.g. a relayed gossip)
    map_capacity: Any = field(default=None, compare=False)
    JAVA = "io.scalecube.cluster.transport.api.Message"

    def header(self, name):
        return dict(self.headers).get(name)

    def write_external(self, out):  # Message.java:206-215
        hs = java_hashmap_order(self.headers, self.map_capacity)
        out.write_int(len(hs))
        for k, v in hs:
            out.write_utf(k)
            out.write_utf("null" if v is None else v)
        out.write_object(self.data)

    @classmethod
    def read_external(cls, inp):  # Message.java:218-230
        hs = []
        n = inp.read_int()
        for _ in range(n):
            k, v = inp.read_utf(), inp.read_utf()
            hs.append((k, None if v == "null" else v))
        return cls(tuple(hs), inp.read_object(), n)


@dataclass(frozen=True)
class Gossip:
    gossiper_id: str
    message: Message
    sequence_id: int
    JAVA = "io.scalecube.cluster.gossip.Gossip"

    def write_external(self, out):
        out.write_utf(self.gossiper_id)
        out.write_object(self.message)
        out.write_long(self.sequence_id)

    @classmethod
    def read_external(cls, inp):
        g = inp.read_utf()
        m = inp.read_object()
        return cls(g, m, inp.read_long())


@dataclass(frozen=True)
class GossipRequest:
    gossips: tuple
    sender: str  # GossipRequest.from
    JAVA = "io.scalecube.cluster.gossip.GossipRequest"

    def write_external(self, out):
        out.write_int(len(self.gossips))
        for g in self.gossips:
            out.write_object(g)
        out.write_utf(self.sender)

    @classmethod
    def read_external(cls, inp):
        gs = tuple(inp.read_object() for _ in range(inp.read_int()))
        return cls(gs, inp.read_utf())


@dataclass(frozen=True)
class PingData:
    sender: Member
    target: Member
    original_issuer: Member | None = None
    gone: bool | None = None  # AckType: None (a ping), False DEST_OK, True DEST_GONE
    JAVA = "io.scalecube.cluster.fdetector.PingData"

    def write_external(self, out):
        out.write_object(self.sender)
        out.write_object(self.target)
        out.write_object(self.original_issuer)
        out.write_object(None if self.gone is None else ack_type(self.gone))

    @classmethod
    def read_external(cls, inp):
        f, t, o, a = inp.read_object(), inp.read_object(), inp.read_object(), inp.read_object()
        return cls(f, t, o, None if a is None else a.name == "DEST_GONE")


@dataclass(frozen=True)
class GetMetadataRequest:
    member: Member
    JAVA = "io.scalecube.cluster.metadata.GetMetadataRequest"

    def write_external(self, out):
        out.write_object(self.member)

    @classmethod
    def read_external(cls, inp):
        return cls(inp.read_object())


@dataclass(frozen=True)
class GetMetadataResponse:
    member: Member
    metadata: bytes
    JAVA = "io.scalecube.cluster.metadata.GetMetadataResponse"

    def write_external(self, out):
        out.write_object(self.member)
        out.write_int(len(self.metadata))
        out.write(self.metadata)

    @classmethod
    def read_external(cls, inp):
        m = inp.read_object()
        return cls(m, inp.read_fully(inp.read_int()))


EXTERNALIZABLE = {c.JAVA: c for c in (Member, MembershipRecord, SyncData, Message, Gossip, GossipRequest, PingData,
                                      GetMetadataRequest, GetMetadataResponse)}


# ------------------------------------------------------------------------------- java.util.HashMap order
def java_string_hash(s: str) -> int:
    """String.hashCode over UTF-16 code units, as a signed 32-bit int"""
    h = 0
    for (cu,) in struct.iter_unpack(">H", s.encode("utf-16-be")):
        h = (31 * h + cu) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


def java_hashmap_order(items, initial_capacity=None) -> list:
    """Iteration order of a java.util.HashMap filled by put() in the given order: by bucket index
    (h ^ h >>> 16) & (capacity - 1), then insertion order (a resize keeps the relative order inside
    each bucket).  Re-putting a key keeps its place.  `initial_capacity` None: `new HashMap<>()`
    (Message.Builder, Message.java:234: a 16-bucket table at the first put); n: `new HashMap<>(n)`
    (Message.readExternal, :221: tableSizeFor(n) buckets).  The table doubles when the size passes
    0.75 of the capacity (HashMap.putVal / resize)."""
    seen, order = {}, []
    for k, v in items:
        if k not in seen:
            order.append(k)
        seen[k] = v
    if initial_capacity is None:
        cap = 16
    else:
        cap = 1
        while cap < initial_capacity:  # tableSizeFor
            cap *= 2
    thr = int(cap * 0.75)
    for size in range(1, len(order) + 1):
        if size > thr:
            cap *= 2
            thr = int(cap * 0.75)

    def bucket(k):
        h = java_string_hash(k) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)
    return [(k, seen[k]) for _, k in sorted(((bucket(k), i), k) for i, k in enumerate(order))]


# ------------------------------------------------------------------------------- output stream
def _mutf8(s: str) -> bytes:
    """Java modified UTF-8 (DataOutput.writeUTF body): NUL as 0xC0 0x80, supplementary characters
    as two 3-byte surrogates"""
    out = bytearray()
    for (cu,) in struct.iter_unpack(">H", s.encode("utf-16-be")):
        if 0x0001 <= cu <= 0x007F:
            out.append(cu)
        elif cu <= 0x07FF:
            out += bytes((0xC0 | (cu >> 6), 0x80 | (cu & 0x3F)))
        else:
            out += bytes((0xE0 | (cu >> 12), 0x80 | ((cu >> 6) & 0x3F), 0x80 | (cu & 0x3F)))
    return bytes(out)


class ObjectOutput:
    """java.io.ObjectOutputStream (protocol version 2) for the classes above."""

    def __init__(self):
        self.buf = bytearray(struct.pack(">HH", STREAM_MAGIC, STREAM_VERSION))
        self.block = bytearray()  # pending block data
        self.block_mode = True    # the constructor leaves the stream in block-data mode
        self.handles: dict = {}   # identity key -> handle
        self.next_handle = BASE_HANDLE

    # -- primitive data (block-data mode: buffered, emitted in blocks of up to 1,024 bytes)
    def _data(self, b: bytes) -> None:
        if not self.block_mode:
            self.buf += b
            return
        for x in b:
            self.block.append(x)
            if len(self.block) == MAX_BLOCK:
                self._flush_block()

    def _flush_block(self) -> None:
        n = len(self.block)
        if n == 0:
            return
        self.buf += bytes((TC_BLOCKDATA, n)) if n <= 0xFF else bytes((TC_BLOCKDATALONG,)) + struct.pack(">i", n)
        self.buf += self.block
        self.block = bytearray()

    def write_int(self, v): self._data(struct.pack(">i", v))
    def write_long(self, v): self._data(struct.pack(">q", v))
    def write_short(self, v): self._data(struct.pack(">h", v))
    def write_boolean(self, v): self._data(b"\x01" if v else b"\x00")
    def write(self, b: bytes): self._data(bytes(b))

    def write_utf(self, s: str) -> None:
        body = _mutf8(s)
        if len(body) > 0xFFFF:
            raise ValueError("UTF encoding longer than 65,535 bytes")
        self._data(struct.pack(">H", len(body)) + body)

    # -- raw (non-block) structure
    def _raw_utf(self, s: str) -> None:
        body = _mutf8(s)
        self.buf += struct.pack(">H", len(body)) + body

    def _assign(self, key) -> None:
        self.handles[key] = self.next_handle
        self.next_handle += 1

    def _ref(self, key) -> bool:
        h = self.handles.get(key)
        if h is None:
            return False
        self.buf += bytes((TC_REFERENCE,)) + struct.pack(">i", h)
        return True

    def _class_desc(self, name: str, suid: int, flags: int, super_desc=None) -> None:
        if self._ref(("desc", name)):
            return
        self.buf.append(TC_CLASSDESC)
        self._assign(("desc", name))
        self._raw_utf(name)
        self.buf += struct.pack(">qBh", suid, flags, 0)  # serialVersionUID, flags, no fields
        self.buf.append(TC_ENDBLOCKDATA)                  # annotateClass: nothing
        if super_desc is None:
            self.buf.append(TC_NULL)
        else:
            self._class_desc(*super_desc)

    def write_object(self, obj) -> None:
        was = self.block_mode
        if was:  # ObjectOutputStream.writeObject0 leaves block-data mode for the object itself
            self._flush_block()
            self.block_mode = False
        if obj is None:
            self.buf.append(TC_NULL)
        elif isinstance(obj, JavaEnum):  # writeEnum: descriptor chain, handle, name
            if not self._ref(("enum", obj.cls, obj.name)):
                self.buf.append(TC_ENUM)
                self._class_desc(obj.cls, 0, SC_SERIALIZABLE | SC_ENUM, ("java.lang.Enum", 0, SC_SERIALIZABLE | SC_ENUM))
                self._assign(("enum", obj.cls, obj.name))
                self._write_string(obj.name)
        elif isinstance(obj, str):
            self._write_string(obj, shared=False)
        elif type(obj).__name__ in {c.__name__ for c in EXTERNALIZABLE.values()}:
            self.buf.append(TC_OBJECT)  # writeOrdinaryObject -> writeExternalData (protocol 2)
            self._class_desc(obj.JAVA, 1, SC_EXTERNALIZABLE | SC_BLOCK_DATA)
            self._assign(("obj", id(obj), len(self.handles)))  # every instance is a new object
            self.block_mode = True
            obj.write_external(self)
            self._flush_block()
            self.block_mode = False
            self.buf.append(TC_ENDBLOCKDATA)
        else:
            raise TypeError(f"no wire format for {type(obj).__name__}")
        self.block_mode = was

    def _write_string(self, s: str, shared: bool = True) -> None:
        body = _mutf8(s)
        self.buf += bytes((TC_STRING,)) + struct.pack(">H", len(body)) + body if len(body) <= 0xFFFF else \
            bytes((TC_LONGSTRING,)) + struct.pack(">q", len(body)) + body
        self._assign(("str", id(s), len(self.handles)))

    def getvalue(self) -> bytes:
        self._flush_block()
        return bytes(self.buf)


# ------------------------------------------------------------------------------- input stream
class ObjectInput:
    """java.io.ObjectInputStream for the same subset (reads what ObjectOutput writes)."""

    def __init__(self, b: bytes):
        self.b, self.p = bytes(b), 0
        magic, ver = struct.unpack_from(">HH", self.b, 0)
        if magic != STREAM_MAGIC or ver != STREAM_VERSION:
            raise ValueError("not a Java serialization stream")
        self.p = 4
        self.block_left = 0
        self.block_mode = True
        self.handles: list = []

    def _raw(self, n) -> bytes:
        if self.p + n > len(self.b):
            raise EOFError("truncated stream")
        out = self.b[self.p:self.p + n]
        self.p += n
        return out

    def _data(self, n) -> bytes:
        if not self.block_mode:
            return self._raw(n)
        out = bytearray()
        while n:
            if self.block_left == 0:
                tc = self._raw(1)[0]
                if tc == TC_BLOCKDATA:
                    self.block_left = self._raw(1)[0]
                elif tc == TC_BLOCKDATALONG:
                    self.block_left = struct.unpack(">i", self._raw(4))[0]
                else:
                    raise ValueError(f"expected block data, got {tc:#x}")
            k = min(n, self.block_left)
            out += self._raw(k)
            self.block_left -= k
            n -= k
        return bytes(out)

    def read_int(self): return struct.unpack(">i", self._data(4))[0]
    def read_long(self): return struct.unpack(">q", self._data(8))[0]
    def read_boolean(self): return self._data(1) != b"\x00"
    def read_fully(self, n): return self._data(n)

    def read_utf(self) -> str:
        n = struct.unpack(">H", self._data(2))[0]
        return _demutf8(self._data(n))

    def _raw_utf(self) -> str:
        n = struct.unpack(">H", self._raw(2))[0]
        return _demutf8(self._raw(n))

    def _class_desc(self):
        tc = self._raw(1)[0]
        if tc == TC_NULL:
            return None
        if tc == TC_REFERENCE:
            return self.handles[struct.unpack(">i", self._raw(4))[0] - BASE_HANDLE]
        if tc != TC_CLASSDESC:
            raise ValueError(f"expected a class descriptor, got {tc:#x}")
        slot = len(self.handles)
        self.handles.append(None)
        name = self._raw_utf()
        suid, flags, nfields = struct.unpack(">qBh", self._raw(11))
        if nfields != 0:
            raise ValueError(f"{name}: serializable fields are outside this codec")
        if self._raw(1)[0] != TC_ENDBLOCKDATA:
            raise ValueError(f"{name}: class annotations are outside this codec")
        desc = {"name": name, "suid": suid, "flags": flags}
        self.handles[slot] = desc
        desc["super"] = self._class_desc()
        return desc

    def read_object(self):
        was = self.block_mode
        if was and self.block_left:
            raise ValueError("unread block data before an object")
        self.block_mode = False
        tc = self._raw(1)[0]
        if tc == TC_NULL:
            obj = None
        elif tc == TC_REFERENCE:
            obj = self.handles[struct.unpack(">i", self._raw(4))[0] - BASE_HANDLE]
        elif tc == TC_ENUM:
            desc = self._class_desc()
            slot = len(self.handles)
            self.handles.append(None)
            name = self.read_object()
            obj = JavaEnum(desc["name"], name)
            self.handles[slot] = obj
        elif tc == TC_STRING:
            obj = self._raw_utf()
            self.handles.append(obj)
        elif tc == TC_OBJECT:
            desc = self._class_desc()
            if not desc["flags"] & SC_EXTERNALIZABLE or not desc["flags"] & SC_BLOCK_DATA:
                raise ValueError(f"{desc['name']}: only Externalizable (protocol 2) objects are decoded")
            cls = EXTERNALIZABLE.get(desc["name"])
            if cls is None:
                raise ValueError(f"unknown class {desc['name']}")
            slot = len(self.handles)
            self.handles.append(None)
            self.block_mode, self.block_left = True, 0
            obj = cls.read_external(self)
            if self.block_left or self._raw(1)[0] != TC_ENDBLOCKDATA:
                raise ValueError(f"{desc['name']}: data left after readExternal")
            self.handles[slot] = obj
        else:
            raise ValueError(f"unsupported type code {tc:#x}")
        self.block_mode = was
        return obj


def _demutf8(b: bytes) -> str:
    cus, i = [], 0
    while i < len(b):
        x = b[i]
        if x < 0x80:
            cus.append(x)
            i += 1
        elif x >> 5 == 0x6:
            cus.append(((x & 0x1F) << 6) | (b[i + 1] & 0x3F))
            i += 2
        else:
            cus.append(((x & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F))
            i += 3
    return struct.pack(f">{len(cus)}H", *cus).decode("utf-16-be", errors="surrogatepass")


# ------------------------------------------------------------------------------- codec
def serialize(message: Message) -> bytes:
    """JdkMessageCodec.serialize (:20-25)"""
    out = ObjectOutput()
    message.write_external(out)
    return out.getvalue()


def deserialize(b: bytes) -> Message:
    """JdkMessageCodec.deserialize (:11-18)"""
    inp = ObjectInput(b)
    return Message.read_external(inp)


# ------------------------------------------------------------------------------- engine bridge
@dataclass
class Directory:
    """Java identities of the engine's member slots: id, address (host:port) and namespace."""
    ids: list
    addresses: list
    namespaces: list = field(default_factory=list)

    @classmethod
    def local(cls, n: int, host: str = "localhost", base_port: int = 4800, namespace: str = "default"):
        return cls([f"{m:08x}" for m in range(n)], [f"{host}:{base_port + m}" for m in range(n)], [namespace] * n)

    def member(self, m: int) -> Member:
        return Member(self.ids[m], self.addresses[m], self.namespaces[m] if self.namespaces else "default")


def sync_message(engine, viewer: int, directory: Directory, ack: bool = False, cid: str | None = None) -> Message:
    """The SYNC (or SYNC_ACK) a simulated member sends: its whole membership table (prepareSyncDataMsg,
    MembershipProtocolImpl.java:485-489) from the engine's view row of `viewer`."""
    row = engine.read_view(viewer)
    recs = []
    for s in range(len(row)):
        cell = int(row[s])
        if (cell >> 34) & 1:  # in the table
            recs.append(MembershipRecord(directory.member(s), (cell >> 32) & 3, cell & 0xFFFFFFFF))
    hs = [(HEADER_QUALIFIER, SYNC_ACK if ack else SYNC)]
    if cid is not None:
        hs.append((HEADER_CORRELATION_ID, cid))
    hs.append((HEADER_SENDER, directory.addresses[viewer]))
    return Message(tuple(hs), SyncData(tuple(recs)))


def engine_records(message: Message, directory: Directory) -> list:
    """The records of a decoded SYNC / SYNC_ACK (its SyncData, in list order) as (member slot, status,
    incarnation) for swim_ingest_sync (Engine.ingest_sync); members the directory does not know are
    left out (the engine simulates a fixed set of slots)."""
    index = {mid: m for m, mid in enumerate(directory.ids)}
    out = []
    for r in message.data.membership:
        m = index.get(r.member.id)
        if m is not None:
            out.append((m, r.status, r.incarnation))
    return out


def gossip_request(engine, sender: int, gossips: list, directory: Directory) -> Message:
    """A GOSSIP_REQ of a simulated member carrying membership gossips (GossipProtocolImpl.java:288-300,
    MembershipProtocolImpl.java:847-852), `gossips` = (gossiper slot, sequence id, subject slot, status,
    incarnation) tuples, e.g. from engine.read_gossips(sender)."""
    out = []
    for g, seq, subj, st, inc in gossips:
        rec = MembershipRecord(directory.member(subj), st, inc)
        out.append(Gossip(directory.ids[g], Message(((HEADER_QUALIFIER, MEMBERSHIP_GOSSIP),), rec), seq))
    return Message(((HEADER_QUALIFIER, GOSSIP_REQ), (HEADER_SENDER, directory.addresses[sender])),
                   GossipRequest(tuple(out), directory.ids[sender]))
