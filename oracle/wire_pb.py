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


def unmarshal(b: bytes):
    m = epoch_tree_object_class()()
    m.ParseFromString(b)
    return m
