"""EpochTreeObject (datap/data.proto:60-68) via the official protobuf runtime -- TEST
INFRASTRUCTURE ONLY (the checker for the device wire encoder/decoder, mydatastore_amd/csrc/wire.hip).

No protoc in the image, so the message descriptor is built field by field from the reference
schema; tests/test_wire.py checks it against datap/data.proto when the reference is present.
protobuf-python and protobuf-go (google.golang.org/protobuf v1.30, main/go.mod) both emit proto3
fields in field-number order, omit zero scalars and pack repeated int32, so this runtime's bytes are
the bytes proto.Marshal produces at main/manager.go:1045.
"""
from functools import lru_cache

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

FIELDS = [  # (name, number, type, repeated) -- datap/data.proto:60-68
    ("partition", 1, "TYPE_INT32", False),
    ("lower_epoch", 2, "TYPE_INT64", False),
    ("upper_epoch", 3, "TYPE_INT64", False),
    ("buckets", 4, "TYPE_BYTES", True),
    ("buckets_size", 5, "TYPE_INT32", True),
    ("valid", 6, "TYPE_BOOL", False),
    ("items", 7, "TYPE_INT32", False),
]


@lru_cache(None)
def epoch_tree_object_class():
    T = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="datap_epoch_tree.proto", package="datap", syntax="proto3")
    m = fdp.message_type.add(name="EpochTreeObject")
    for name, num, typ, rep in FIELDS:
        m.field.add(name=name, number=num, type=getattr(T, typ),
                    label=T.LABEL_REPEATED if rep else T.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("datap.EpochTreeObject"))


def marshal(partition, lower, upper, digests, sizes, valid=False, items=None):
    """proto.Marshal(MerkleTreeToPartitionEpochObject(tree(digests, sizes), ...)): leaves follow
    tree.Leafs (odd B repeats the last bucket); items = leaf-size sum (int32 wrap) unless given."""
    from oracle.oracle import encode_int64_to_bytes, _int32
    d, s = list(digests), list(sizes)
    if len(d) % 2 == 1:
        d.append(d[-1])
        s.append(s[-1])
    if items is None:
        items = 0
        for x in s:
            items = _int32(items + x)
    msg = epoch_tree_object_class()(partition=partition, lower_epoch=lower, upper_epoch=upper,
                                     buckets=[encode_int64_to_bytes(_i64(x)) for x in d],
                                     buckets_size=s, valid=valid, items=items)
    return msg.SerializeToString()


def _i64(x):
    x = int(x) & 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >= 1 << 63 else x


class WireError(ValueError):
    """proto.Unmarshal error (protobuf-go returns errDecode; the peer is skipped)."""


MAX_VALID_NUMBER = (1 << 29) - 1  # protowire.MaxValidNumber
RECURSION_LIMIT = 10000           # protowire.DefaultRecursionLimit


def _varint(b, pos):
    """protowire.ConsumeVarint (google.golang.org/protobuf v1.30, encoding/protowire/wire.go):
    at most 10 bytes, and the 10th must be 0 or 1 (errCodeOverflow)."""
    v = 0
    for i in range(10):
        if pos + i >= len(b):
            raise WireError("truncated varint")
        y = b[pos + i]
        if i == 9:
            if y >= 2:
                raise WireError("varint overflow")
            return v | (y << 63), pos + 10
        v |= (y & 0x7F) << (7 * i)
        if y < 0x80:
            return v, pos + i + 1
    raise AssertionError


def _tag(b, pos):
    """protowire.ConsumeTag: DecodeTag maps x>>3 > MaxInt32 to -1; numbers < 1 fail."""
    v, pos = _varint(b, pos)
    num = -1 if (v >> 3) > 0x7FFFFFFF else v >> 3
    if num < 1:
        raise WireError("invalid field number")
    return num, v & 7, pos


def _skip(b, pos, num, typ, depth):
    """protowire.consumeFieldValueD: the value of an unknown field (groups recursively, the end
    tag's number must match; depth-limited); wire types 6/7 and a stray end group fail."""
    if typ == 0:
        return _varint(b, pos)[1]
    if typ in (1, 5):
        n = 8 if typ == 1 else 4
        if len(b) - pos < n:
            raise WireError("truncated fixed")
        return pos + n
    if typ == 2:
        n, pos = _varint(b, pos)
        if n > len(b) - pos:
            raise WireError("truncated bytes")
        return pos + n
    if typ == 3:
        # consumeFieldValueD's recursion, unrolled onto an explicit stack (Python's own stack is
        # shallower than the 10,000 levels Go allows): each open group keeps (number, depth); a
        # group is entered only with depth >= 0, so at most RECURSION_LIMIT + 1 levels nest
        stack = [(num, depth)]
        while stack:
            if stack[-1][1] < 0:
                raise WireError("recursion")
            num2, typ2, pos = _tag(b, pos)
            if typ2 == 4:
                if num2 != stack[-1][0]:
                    raise WireError("end group mismatch")
                stack.pop()
            elif typ2 == 3:
                stack.append((num2, stack[-1][1] - 1))
            else:
                pos = _skip(b, pos, num2, typ2, 0)
        return pos
    raise WireError("end group / reserved wire type")


class _Object:
    __slots__ = ("partition", "lower_epoch", "upper_epoch", "buckets", "buckets_size", "valid", "items")


def _s32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def unmarshal(b: bytes):
    """proto.Unmarshal of an EpochTreeObject as protobuf-go v1.30 (main/go.mod:15) decodes it
    (internal/impl/decode.go unmarshalPointer + the proto3 field coders): top-level field numbers
    in [1, 2^29-1]; a known field with another wire type is an unknown field; unknown fields are
    skipped by protowire.ConsumeFieldValue; int32 = int32(varint), int64 = int64(varint), bool =
    varint != 0; bytes and repeated int32 (packed or not) append. Raises WireError where Go
    returns an error. (The upb runtime agrees on well-formed objects -- tests/test_wire.py -- but
    accepts a 10th varint byte >= 2, which Go rejects.)"""
    b = bytes(b)
    m = _Object()
    m.partition = m.lower_epoch = m.upper_epoch = m.items = 0
    m.valid = False
    m.buckets, m.buckets_size = [], []
    pos = 0
    while pos < len(b):
        v, pos = _varint(b, pos)
        num, typ = v >> 3, v & 7
        if num < 1 or num > MAX_VALID_NUMBER:
            raise WireError("invalid field number")
        if typ == 0 and num in (1, 2, 3, 6, 7):
            x, pos = _varint(b, pos)
            if num == 1:
                m.partition = _s32(x)
            elif num == 2:
                m.lower_epoch = _i64(x)
            elif num == 3:
                m.upper_epoch = _i64(x)
            elif num == 6:
                m.valid = x != 0
            else:
                m.items = _s32(x)
        elif typ == 2 and num == 4:
            n, pos = _varint(b, pos)
            if n > len(b) - pos:
                raise WireError("truncated bytes")
            m.buckets.append(b[pos:pos + n])
            pos += n
        elif typ == 2 and num == 5:
            n, pos = _varint(b, pos)
            if n > len(b) - pos:
                raise WireError("truncated packed")
            end = pos + n
            while pos < end:
                x, pos = _varint(b[:end], pos)
                m.buckets_size.append(_s32(x))
        elif typ == 0 and num == 5:
            x, pos = _varint(b, pos)
            m.buckets_size.append(_s32(x))
        else:
            pos = _skip(b, pos, num, typ, RECURSION_LIMIT)
    return m


def unmarshal_upb(b: bytes):
    """The protobuf-python (upb) runtime's parse, kept as a cross-check of unmarshal()."""
    m = epoch_tree_object_class()()
    m.ParseFromString(b)
    return m
