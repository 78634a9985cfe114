"""EpochTreeObject wire bytes: device encoder/decoder (mydatastore_amd/csrc/wire.hip) against the
official protobuf runtime (oracle/wire_pb.py)."""
import re
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O
from oracle import wire_pb
from tests.datasets import synth_arrays

REF_PROTO = Path("/root/reference/datap/data.proto")


def test_descriptor_matches_reference_schema():
    if not REF_PROTO.exists():
        pytest.skip("reference not mounted (GPU box)")
    text = REF_PROTO.read_text()
    body = re.search(r"message EpochTreeObject\s*\{(.*?)\}", text, re.S).group(1)
    fields = re.findall(r"(repeated\s+)?(\w+)\s+(\w+)\s*=\s*(\d+)\s*;", body)
    got = [(name, int(num), "TYPE_" + typ.upper(), bool(rep)) for rep, typ, name, num in fields]
    assert got == wire_pb.FIELDS


def test_oracle_roundtrip_testmerkletreeraw(golden):
    fix = golden("testmerkletreeraw_n100.json")
    tr = fix["trees"]["0_3"]
    b = wire_pb.marshal(0, 0, 3, tr["digests"], tr["sizes"])
    m = wire_pb.unmarshal(b)
    assert [x.hex() for x in m.buckets] == tr["object_buckets"] and m.items == tr["items"]
    assert b[:2] == bytes([0x18, 0x03])  # partition 0 and lower_epoch 0 omitted (proto3)


@pytest.mark.gpu
def test_encode_matches_protobuf(engine, golden, coracle):
    rng = np.random.default_rng(31)
    for case in golden("synth_cases.json"):
        P, B = case["P"], case["B"]
        dg = np.array(case["digest"], np.uint64)
        sz = np.array(case["size"], np.int32)
        parts = np.arange(P, dtype=np.int32) * 3 - 2       # includes 0 and a negative id
        valid = (np.arange(P) % 2).astype(np.uint8)
        got = engine.encode_objects(B, dg, sz, parts, 7, 8, valid)
        for p in range(P):
            want = wire_pb.marshal(int(parts[p]), 7, 8, case["digest"][p * B:(p + 1) * B],
                                   case["size"][p * B:(p + 1) * B], bool(valid[p]))
            assert got[p] == want, (case["name"], p)
            assert wire_pb.unmarshal(got[p]).items == case["items"][p]
    # extremes: negative sizes/items (10-byte varints), int64 epochs, B = 1
    for B in (1, 2, 3, 64, 1000):
        dg = rng.integers(0, 2**64 - 1, 2 * B, dtype=np.uint64)
        sz = rng.integers(-2**31, 2**31 - 1, 2 * B, dtype=np.int64).astype(np.int32)
        items = np.array([-7, 2**31 - 1], np.int32)
        got = engine.encode_objects(B, dg, sz, np.array([-1, 2**31 - 1], np.int32), -(2**40), 2**62,
                                    None, items)
        for t in range(2):
            want = wire_pb.marshal([-1, 2**31 - 1][t], -(2**40), 2**62, dg[t * B:(t + 1) * B].tolist(),
                                   sz[t * B:(t + 1) * B].tolist(), False, int(items[t]))
            assert got[t] == want, B
    # objects without buckets (built field by field, main/manager_test.go:245-287)
    parts = np.array([0, 1, -3], np.int32)
    valid = np.array([1, 0, 1], np.uint8)
    items = np.array([0, 5, -1], np.int32)
    got = engine.encode_objects(0, np.zeros(0, np.uint64), np.zeros(0, np.int32), parts, 2, 0, valid,
                                items, n_objects=3)
    for t in range(3):
        want = wire_pb.marshal(int(parts[t]), 2, 0, [], [], bool(valid[t]), int(items[t]))
        assert got[t] == want, t
        m = wire_pb.unmarshal(got[t])
        assert len(m.buckets) == 0 and m.valid == bool(valid[t])


@pytest.mark.gpu
def test_decode_matches_protobuf(engine):
    import mydatastore_amd as mde
    rng = np.random.default_rng(32)
    cls = wire_pb.epoch_tree_object_class()
    objs, exp = [], []
    for B in (1, 2, 5, 30, 64, 200):
        d = rng.integers(0, 999999, B).tolist()
        s = rng.integers(0, 500, B).tolist()
        b = wire_pb.marshal(int(rng.integers(-3, 9)), 4, 5, d, s, bool(B % 2), None)
        objs.append(b)
        exp.append(wire_pb.unmarshal(b))
    # sizes shorter than buckets (read as 0), unknown fields, fields out of order, unpacked sizes
    m = cls(partition=9, buckets=[O.encode_int64_to_bytes(5)] * 4, buckets_size=[1, 2])
    odd = m.SerializeToString() + bytes([0x48, 0x05, 0x52, 0x02, 0xAA, 0xBB])  # fields 9 and 10
    odd = bytes([0x38, 0x07]) + odd + bytes([0x28, 0x0B])  # items first; an unpacked size element
    objs.append(odd)
    got = engine.decode_objects(objs, cap=256)
    for g, e in zip(got[:-1], exp):
        assert g["partition"] == e.partition and g["lower"] == e.lower_epoch and g["upper"] == e.upper_epoch
        assert g["valid"] == e.valid and g["items"] == e.items
        assert g["digest"] == [int.from_bytes(x, "little") for x in e.buckets]
        assert g["size"] == list(e.buckets_size)
    assert got[-1]["partition"] == 9 and got[-1]["items"] == 7
    assert got[-1]["digest"] == [5] * 4 and got[-1]["size"] == [1, 2, 11, 0]
    # a 7-byte bucket hash (DecodeBytesToInt64 error), truncation, capacity
    bad = cls(buckets=[b"\0" * 7]).SerializeToString()
    trunc = objs[3][:-1]  # cuts the trailing items varint mid-field
    res = engine.decode_objects([bad, trunc], cap=256)
    assert res[0] == mde.MDE_E_DECODE and res[1] == mde.MDE_E_DECODE
    assert engine.decode_objects([objs[5]], cap=8)[0] == mde.MDE_E_CAPACITY


@pytest.mark.gpu
def test_wire_roundtrip_rebuilds_same_tree(engine, golden, coracle):
    """Peer path: encode -> decode -> EpochTreeObjectToMerkleTree on device == original root."""
    case = next(c for c in golden("synth_cases.json") if c["name"] == "b64_1k")
    P, B = case["P"], case["B"]
    objs = engine.encode_objects(B, np.array(case["digest"], np.uint64), np.array(case["size"], np.int32),
                                 np.arange(P, dtype=np.int32), 1, 2)
    dec = engine.decode_objects(objs, cap=B)
    d = np.array([x for o in dec for x in o["digest"]], np.uint64)
    roots, _ = engine.tree_from_digests(d, B)
    assert [roots[32 * p:32 * p + 32].tobytes().hex() for p in range(P)] == case["root"]


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


@pytest.mark.gpu
def test_decode_wave_runs_and_hostile_lengths(engine):
    """The wave-parallel decoder's run boundaries (bucket runs and packed-size windows of 64,
    capacity inside a run, a non-canonical entry splitting a run, 10-byte negative sizes, objects
    above the 8 KiB LDS stage) and hostile lengths that must fail, not wrap (a length field near
    2^64 once moved the cursor backwards: an endless parse)."""
    import mydatastore_amd as mde
    rng = np.random.default_rng(64)
    cls = wire_pb.epoch_tree_object_class()
    objs, exp = [], []
    for B in (63, 64, 65, 127, 128, 129, 700, 1000):
        d = rng.integers(0, 999999, B).tolist()
        s = rng.integers(-2**31, 2**31, B).tolist()  # 5- and 10-byte varints
        b = wire_pb.marshal(3, 4, 5, d, s, True, None)
        objs.append(b)
        exp.append(wire_pb.unmarshal(b))
    assert len(objs[-1]) > 8 << 10  # parsed from global memory, not the LDS stage
    got = engine.decode_objects(objs, cap=1024)
    for g, e in zip(got, exp):
        assert g["digest"] == [int.from_bytes(x, "little") for x in e.buckets]
        assert g["size"] == list(e.buckets_size)
        assert g["valid"] == e.valid and g["partition"] == e.partition
    # capacity reached inside a run (entry cap + 1 fails), for several window offsets
    for B, cap in ((65, 64), (129, 100), (700, 640), (64, 64)):
        r = engine.decode_objects([objs[(63, 64, 65, 127, 128, 129, 700, 1000).index(B)]], cap=cap)[0]
        assert (r == mde.MDE_E_CAPACITY) if B > cap else isinstance(r, dict)


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [16, 1024])
def test_decode_split_run_and_malformed_varints(engine, cap):
    """Both decode_kernel instantiations (64-wide windows for cap <= 64, 256-wide above): a
    bucket run split by a non-canonical entry, and the malformed varints and wrapping lengths
    that must fail."""
    import mydatastore_amd as mde
    rng = np.random.default_rng(64)
    cls = wire_pb.epoch_tree_object_class()
    # a run split by a non-canonical entry: overlong key varint 0xA2 0x00 (= field 4, wire type 2)
    ent = [int(x) for x in rng.integers(0, 999999, 6)]
    body = b"".join(b"\x22\x08" + v.to_bytes(8, "little") for v in ent[:3])
    body += b"\xa2\x00\x08" + ent[3].to_bytes(8, "little")
    body += b"".join(b"\x22\x08" + v.to_bytes(8, "little") for v in ent[4:])
    pk = b"".join(_varint(x) for x in (1, 300, 2**32 - 1))
    split = body + b"\x2a" + _varint(len(pk)) + pk
    g = engine.decode_objects([split], cap=cap)[0]
    assert g["digest"] == ent and g["size"] == [1, 300, -1, 0, 0, 0]
    assert [int.from_bytes(x, "little") for x in cls.FromString(split).buckets] == ent
    # failures: 11-byte size varint, a varint crossing the packed run's end, wrapping lengths
    eleven = b"\x2a\x0b" + b"\xff" * 10 + b"\x01"
    cross = b"\x2a\x02\x01\x80\x01"
    wrap_unknown = b"\x08\x01\x0a" + _varint(2**64 - 12)  # field 1, wire type 2: skipped
    wrap_bucket = b"\x22" + _varint(2**64 - 1)
    wrap_packed = b"\x2a" + _varint(2**64 - 11) + b"\x01"
    res = engine.decode_objects([eleven, cross, wrap_unknown, wrap_bucket, wrap_packed], cap=cap)
    assert res == [mde.MDE_E_DECODE] * 5


GO_RULE_CASES = {  # object bytes -> True when protobuf-go v1.30 proto.Unmarshal accepts them
    "field0": (b"\x00\x05", False),
    "varint_10th_byte_2": (b"\x08" + b"\xff" * 9 + b"\x02", False),  # upb accepts; Go overflows
    "varint_10th_byte_1": (b"\x08" + b"\xff" * 9 + b"\x01", True),
    "packed_10th_byte_2": (b"\x2a\x0a" + b"\xff" * 9 + b"\x02", False),
    "unknown_group": (b"\x4b\x08\x01\x53\x54\x4c\x08\x05", True),  # 9{1:1 10{}} then partition=5
    "group_end_mismatch": (b"\x4b\x54", False),
    "stray_end_group": (b"\x4c", False),
    "wire_type_6": (b"\x4e", False),
    "wire_type_7": (b"\x4f", False),
    "top_field_2pow29": (b"\x80\x80\x80\x80\x10\x01", False),
    "top_field_max": (b"\xf8\xff\xff\xff\x0f\x01", True),
    "group_inner_field_2pow29": (b"\x4b\x80\x80\x80\x80\x10\x01\x4c", True),  # ConsumeTag: <= MaxInt32
    "group_inner_field_2pow31": (b"\x4b\x80\x80\x80\x80\x80\x02\x01\x4c", False),
    "known_field_other_wire_type": (b"\x0d\x01\x02\x03\x04\x22\x08" + bytes(8), True),
    "bool_2": (b"\x30\x02", True),
    "overlong_key": (b"\x88\x00\x05", True),
}


def test_oracle_unmarshal_go_rules():
    """oracle/wire_pb.unmarshal (the protobuf-go restatement) on the wire-format edge cases, and
    agreement with the upb runtime on well-formed objects."""
    for name, (b, ok) in GO_RULE_CASES.items():
        try:
            wire_pb.unmarshal(b)
            got = True
        except wire_pb.WireError:
            got = False
        assert got == ok, name
    assert wire_pb.unmarshal(GO_RULE_CASES["unknown_group"][0]).partition == 5
    # protowire.DefaultRecursionLimit: 10,001 nested unknown groups skip, 10,002 fail
    for d, ok in ((10001, True), (10002, False)):
        deep = b"\x4b" * d + b"\x4c" * d + b"\x08\x05"
        try:
            got = wire_pb.unmarshal(deep).partition == 5
        except wire_pb.WireError:
            got = False
        assert got == ok, d
    assert wire_pb.unmarshal(GO_RULE_CASES["bool_2"][0]).valid
    rng = np.random.default_rng(9)
    for B in (0, 1, 2, 7, 64, 129):
        d = rng.integers(0, 999999, B).tolist()
        s = rng.integers(-2**31, 2**31, B).tolist()
        b = wire_pb.marshal(int(rng.integers(-5, 5)), 3, 4, d, s, bool(B % 2))
        a, u = wire_pb.unmarshal(b), wire_pb.unmarshal_upb(b)
        for k in ("partition", "lower_epoch", "upper_epoch", "valid", "items"):
            assert getattr(a, k) == getattr(u, k)
        assert list(a.buckets) == list(u.buckets) and list(a.buckets_size) == list(u.buckets_size)


def _expect_decode(obj, cap):
    import mydatastore_amd as mde
    try:
        m = wire_pb.unmarshal(obj)
    except wire_pb.WireError:
        return mde.MDE_E_DECODE
    if any(len(x) != 8 for x in m.buckets):
        return mde.MDE_E_DECODE  # EpochTreeObjectToMerkleTree -> DecodeBytesToInt64
    nb = len(m.buckets)
    if nb > cap:
        return mde.MDE_E_CAPACITY
    return {"partition": m.partition, "lower": m.lower_epoch, "upper": m.upper_epoch, "valid": m.valid,
            "items": m.items, "digest": [int.from_bytes(x, "little") for x in m.buckets],
            "size": (list(m.buckets_size) + [0] * nb)[:nb]}


def _mutate(rng, b):
    b = bytearray(b)
    for _ in range(int(rng.integers(1, 4))):
        op = int(rng.integers(0, 6))
        at = int(rng.integers(0, len(b) + 1))
        if op == 0 and b:      # overwrite a byte
            b[min(at, len(b) - 1)] = int(rng.integers(0, 256))
        elif op == 1:          # insert random bytes
            b[at:at] = bytes(rng.integers(0, 256, int(rng.integers(1, 4))).tolist())
        elif op == 2 and b:    # delete a range
            del b[at:at + int(rng.integers(1, 12))]
        elif op == 3:          # truncate
            del b[at:]
        elif op == 4:          # splice one of the wire-rule cases
            b[at:at] = list(GO_RULE_CASES.values())[int(rng.integers(0, len(GO_RULE_CASES)))][0]
        else:                  # set / clear a continuation bit
            if b:
                b[min(at, len(b) - 1)] ^= 0x80
    return bytes(b)


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [64, 1024])
def test_decode_follows_go_unmarshal(engine, cap):
    """Device decoder vs the protobuf-go restatement: the wire-rule cases, then 3,000 seeded
    mutations (byte overwrites, insertions, deletions, truncations, continuation-bit flips,
    spliced edge cases) of valid objects -- same error class or the same decoded fields. Both
    decode_kernel instantiations: cap 64 (64-wide windows) and cap 1024 (256-wide windows, with
    objects of up to 700 buckets among the mutated bases)."""
    rng = np.random.default_rng(2024 + cap)
    objs = [b for b, _ in GO_RULE_CASES.values()]
    base = []
    for B in (1, 3, 30, 64, 70) + ((130, 300, 700) if cap > 64 else ()):
        d = rng.integers(0, 999999, B).tolist()
        s = rng.integers(-2**31, 2**31, B).tolist() if B % 2 else rng.integers(0, 300, B).tolist()
        base.append(wire_pb.marshal(int(rng.integers(-9, 9)), 6, 7, d, s, bool(B % 2)))
    objs += base
    objs += [_mutate(rng, base[int(rng.integers(0, len(base)))]) for _ in range(3000)]
    got = engine.decode_objects(objs, cap=cap)
    bad = [(i, g, _expect_decode(o, cap)) for i, (g, o) in enumerate(zip(got, objs)) if g != _expect_decode(o, cap)]
    assert not bad, bad[:5]
    n_err = sum(1 for g in got if not isinstance(g, dict))
    assert 300 < n_err < 2900  # the mutations exercise both outcomes


def _tagb(num, wt):
    return _varint((num << 3) | wt)


def _group_walk(rng, targets, sib=0.3, big_numbers=True):
    """Unknown-group nesting that walks through the depths in `targets` (down and up again),
    with random sibling fields (varint, fixed32/64, length-delimited, small closed groups) between
    the tags; returns the bytes (all groups closed when the walk ends at 0) and the open stack."""
    out, stack = bytearray(), []

    def sibling():
        k = int(rng.integers(0, 5))
        n = int(rng.integers(8, 40))
        if k == 0:
            return _tagb(n, 0) + _varint(int(rng.integers(0, 2**40)))
        if k == 1:
            return _tagb(n, 1) + bytes(8)
        if k == 2:
            return _tagb(n, 5) + bytes(4)
        if k == 3:
            return _tagb(n, 2) + _varint(3) + b"abc"
        return _tagb(n, 3) + _tagb(9, 0) + b"\x01" + _tagb(n, 4)

    for t in targets:
        while len(stack) < t:
            if rng.random() < sib:
                out += sibling()
            n = int(rng.integers(1, 2**31)) if (big_numbers and rng.random() < 0.2) else int(rng.integers(1, 16))
            out += _tagb(n, 3)
            stack.append(n)
        while len(stack) > t:
            if rng.random() < sib:
                out += sibling()
            out += _tagb(stack.pop(), 4)
    return bytes(out), stack


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [64, 1024])
def test_decode_deep_unknown_groups_follow_go(engine, cap):
    """Unknown groups nested beyond the decoder's 64-level ring: protobuf-go skips up to 10,001
    levels (protowire.DefaultRecursionLimit) and rejects the 10,002nd; an end tag whose number
    left the ring is matched after a rescan. Straight nests, zig-zag walks with siblings and
    multi-byte field numbers, deep end-number mismatches and truncations: the device decode
    equals the protobuf-go restatement (oracle/wire_pb.py) for both decode_kernel shapes."""
    import mydatastore_amd as mde
    rng = np.random.default_rng(10001 + cap)
    tail = b"\x08\x05\x10\x06\x22\x08" + (1234).to_bytes(8, "little")  # partition 5, lower 6, one bucket
    objs = []
    for d in (63, 64, 65, 129, 1000, 10001, 10002):
        objs.append(_group_walk(rng, [d, 0], sib=0.0, big_numbers=False)[0] + tail)
    for targets in ([200, 50, 300, 0], [70, 3, 140, 65, 66, 0], [5000, 4000, 9000, 100, 0],
                    [10001, 9000, 10001, 0], [10001, 10000, 10002, 0]):
        objs.append(_group_walk(rng, targets)[0] + tail)
    good = [o for o in objs if isinstance(_expect_decode(o, cap), dict)]
    for o in good[:4]:  # a wrong end number deep inside (after a refill) and a truncation
        b = bytearray(o)
        ends = [i for i in range(len(b) - len(tail)) if b[i] & 7 == 4 and b[i] < 0x80 and (i == 0 or b[i - 1] < 0x80)]
        b[ends[len(ends) // 3]] ^= 0x08  # end tag of another number (or field 0)
        objs.append(bytes(b))
        objs.append(o[: len(o) // 2])
    exp = [_expect_decode(o, cap) for o in objs]
    assert sum(isinstance(e, dict) for e in exp) >= 8 and sum(e == mde.MDE_E_DECODE for e in exp) >= 4
    got = engine.decode_objects(objs, cap=cap)
    bad = [(i, len(objs[i]), g if not isinstance(g, dict) else "ok", e if not isinstance(e, dict) else "ok")
           for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not bad, bad


@pytest.mark.gpu
def test_decode_oscillating_deep_groups_stays_linear(engine):
    """a hostile peer object that nests unknown groups past the 64-level ring and then
    oscillates -- down below the ring's lowest level and back up, ~2,000 times -- made the rescan
    decoder quadratic (each dip rescanned the outer group from its first byte: ~10^8 serial varint
    steps for this 270 KB object). With the spill area the decode is linear: the host-buffer
    decode, the async decode (the context's default spill area) and a VerifyEpoch call carrying the
    object as a peer each finish within a wall-clock bound, and equal the protobuf-go restatement.
    Also the same walk with a wrong end number near the end, and a truncation."""
    import time
    import torch
    import mydatastore_amd as mde
    rng = np.random.default_rng(77)
    targets = [70]
    for _ in range(2000):
        targets += [2, 70]
    targets += [0]
    walk, _ = _group_walk(rng, targets, sib=0.0, big_numbers=False)
    tail = b"\x08\x05\x10\x06\x22\x08" + (1234).to_bytes(8, "little")
    good = walk + tail
    bad_end = bytearray(good)
    i = len(walk) - 3
    while bad_end[i] & 7 != 4:
        i -= 1
    bad_end[i] ^= 0x08
    objs = [good, bytes(bad_end), good[: len(walk) // 2]]
    exp = [_expect_decode(o, 64) for o in objs]
    assert isinstance(exp[0], dict) and exp[1] == mde.MDE_E_DECODE and exp[2] == mde.MDE_E_DECODE
    t0 = time.perf_counter()
    got = engine.decode_objects(objs, cap=64)
    t_sync = time.perf_counter() - t0
    assert got == exp
    # async entry point with device buffers (the context's default spill area covers 8 MiB)
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    off = np.zeros(len(objs) + 1, np.uint64)
    off[1:] = np.cumsum([len(o) for o in objs])
    blob = torch.from_numpy(np.frombuffer(b"".join(objs), np.uint8).copy()).to(dev)
    doff = torch.from_numpy(off.view(np.int64)).to(dev)
    n = len(objs)
    outs = [torch.zeros(n, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.int64, device=dev),
            torch.zeros(n, dtype=torch.int64, device=dev), torch.zeros(n * 64, dtype=torch.int64, device=dev),
            torch.zeros(n * 64, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev),
            torch.zeros(n, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.int32, device=dev)]
    t0 = time.perf_counter()
    engine._call("mde_decode_epoch_tree_objects_async", n, mde._ptr(blob), mde._ptr(doff), 64,
                 *(mde._ptr(o) for o in outs))
    engine.synchronize()
    t_async = time.perf_counter() - t0
    nb = outs[7].cpu().tolist()
    assert nb == [1, mde.MDE_E_DECODE, mde.MDE_E_DECODE]
    assert outs[3].cpu().numpy()[0] == 1234 and outs[0].cpu().numpy()[0] == 5
    # VerifyEpoch with the hostile object as a peer beside an agreeing one (B = 1)
    d = np.array([1234], np.uint64)
    z = np.zeros(1, np.int32)
    root, nodes = engine.tree_from_digests(d, 1)
    t0 = time.perf_counter()
    res = engine.verify_epochs(1, d, z, nodes, [[good, bytes(bad_end)]], replica_count=1, epoch=6, partition=[5])
    t_verify = time.perf_counter() - t0
    assert res["valid_count"] == [1] and res["peer_status"][0] == [0, mde.MDE_E_DECODE]
    assert max(t_sync, t_async, t_verify) < 10.0, (t_sync, t_async, t_verify)
