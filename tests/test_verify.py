"""VerifyEpoch's decision step (main/manager.go:1036-1118): mde_verify_epochs against the oracle.

Each partition gets R peer EpochTreeObjects covering the reference's branches: identical peers
(validCount), perturbed peers (diffSet), a perturbed peer marked Valid (validDiff), absent and
malformed objects, non-8-byte bucket hashes (EpochTreeObjectToMerkleTree error), peers with another
bucket count (same depth: diffable; other depth: DifferentMerkleTreeBuckets error), and the odd-B
duplicate leaf whose bucketId differs from the peer's (the "bucketIds dont match" error).
"""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import wire_pb

STATUS = {O.VERIFY_DECODE: -6, O.VERIFY_TREE: -4}


def _peer_objects(rng, B, digests, sizes, p, E):
    """R = 4 peer objects for partition p, chosen by p % 8."""
    d = [int(x) for x in digests]
    s = [int(x) for x in sizes]

    def obj(dd, ss, valid=False, part=p):
        return wire_pb.marshal(part, E, E + 1, dd, ss, valid=valid)

    def perturb(k):
        dd = list(d)
        for b in rng.choice(B, size=min(k, B), replace=False):
            dd[b] = (dd[b] + 1 + int(rng.integers(0, 999997))) % 999999
        return dd

    same = obj(d, s)
    case = p % 8
    if case == 0:    # all agree
        return [same, same, same, same]
    if case == 1:    # two agree, two differ
        return [same, obj(perturb(1), s), same, obj(perturb(3), s)]
    if case == 2:    # one agrees; a differing peer is marked Valid -> validDiff
        return [same, obj(perturb(2), s, valid=True), None, obj(perturb(1), s)]
    if case == 3:    # absent, truncated, garbage, bad hash length
        bad_hash = wire_pb.epoch_tree_object_class()(partition=p, buckets=[b"\x01\x02\x03"] * 2)
        return [None, same[:-1] if len(same) > 1 else b"\x08", b"\xff\xff\xff", bad_hash.SerializeToString()]
    if case == 4:    # other bucket counts (shallower / same depth / deeper), and an empty object
        odd = wire_pb.epoch_tree_object_class()(  # B-1 buckets on the wire, no duplicate appended
            partition=p, buckets=[O.encode_int64_to_bytes(x) for x in d[:-1]]).SerializeToString()
        return [obj(d[:max(B // 2, 1)], s[:max(B // 2, 1)]), odd, obj(d + d + [7], s + s + [1]), b""]
    if case == 5:    # the last bucket differs (odd B: the duplicate leaf's bucketId mismatches)
        dd = list(d)
        dd[-1] = (dd[-1] + 1) % 999999
        return [obj(dd, s), same, obj(dd, s, valid=True), same]
    if case == 6:    # everything differs
        return [obj(perturb(B), s), obj(perturb(B), s), obj(perturb(B), s), obj(perturb(B), s)]
    # missing sizes and another partition/epoch label: only the buckets matter
    leaves = d + d[-1:] if len(d) % 2 else d
    no_sizes = wire_pb.epoch_tree_object_class()(
        partition=p + 100, lower_epoch=E + 5, upper_epoch=E + 9,
        buckets=[O.encode_int64_to_bytes(x) for x in leaves]).SerializeToString()
    return [no_sizes, obj(perturb(1), s), same, None]


def _oracle_verify(B, digests, sizes, peers, replica, E, parts):
    res = []
    for p, row in enumerate(peers):
        t = O.tree_from_digests(digests[p * B:(p + 1) * B], sizes[p * B:(p + 1) * B])
        res.append(O.verify_epoch(t, int(parts[p]), E, row, replica))
    return res


def test_oracle_verify_testmerkletreeraw_relations(golden):
    """Oracle sanity on the TestMerkleTreeRaw scenario: tree[0,3) vs peers {tree[1,3), tree[2,3)}
    -> one empty diff (validCount 1) and one non-empty diff."""
    m = O.Manager(1, 30)
    ts = 0
    for i in range(100):
        ts += 1
        m.set_value(f"key{i}", f"val{i}", 1, ts)
    for i in range(100):
        ts += 1
        m.set_value(f"keyz{i}", f"valz{i}", 2, ts)
    t1, t2, t3 = (m.raw_partition_merkle_tree(0, lo, 3) for lo in (0, 1, 2))
    o2 = O.merkle_tree_to_partition_epoch_object(t2, 0, 1, 3)
    o3 = O.merkle_tree_to_partition_epoch_object(t3, 0, 2, 3)
    enc = [wire_pb.marshal(0, o.lower_epoch, o.upper_epoch, [O.decode_bytes_to_int64(h) for h in o.buckets],
                           o.buckets_size) for o in (o2, o3)]
    r = O.verify_epoch(t1, 0, 0, enc, replica_count=2)
    assert r["valid_count"] == 1 and not r["valid"]
    assert r["status"][0] == 0 and r["status"][1] > 0
    assert r["diff"] == sorted(set(O.different_merkle_tree_buckets(t1, t3)))
    r = O.verify_epoch(t1, 0, 0, enc, replica_count=1)
    assert r["valid"]


@pytest.mark.gpu
@pytest.mark.parametrize("local_nodes", [True, False], ids=["nodes", "digests_only"])
@pytest.mark.parametrize("mode", [0, 1], ids=["fused", "chain"])
@pytest.mark.parametrize("B", [64, 30, 7, 1, 65, 129, 513, 1000, 1024, 2000])
def test_verify_epochs_matches_oracle(engine, B, mode, local_nodes):
    """Both launch shapes (one fused launch; the decode/tree/diff/fold/encode chain) against the
    oracle. B = 2000 exceeds the fused kernel's peer capacity and runs the chain in both modes.
    digests_only: the local trees' nodes are not given (nodes = NULL, the batcher's form); a
    partition builds its tree on the device when a peer of another shape needs it."""
    rng = np.random.default_rng(1000 + B)
    P, E, replica = 16, 41, 2
    digests = rng.integers(0, 999999, size=P * B, dtype=np.uint64)
    sizes = rng.integers(0, 5000, size=P * B).astype(np.int32)
    parts = (np.arange(P) * 7 + 3).astype(np.int32)
    _, nodes = engine.tree_from_digests(digests, B)
    peers = [_peer_objects(rng, B, digests[p * B:(p + 1) * B], sizes[p * B:(p + 1) * B], int(parts[p]), E)
             for p in range(P)]
    engine.set_verify_mode(mode)
    try:
        got = engine.verify_epochs(B, digests, sizes, nodes if local_nodes else None, peers, replica, E,
                                   partition=parts)
    finally:
        engine.set_verify_mode(0)
    want = _oracle_verify(B, digests, sizes, peers, replica, E, parts)
    for p in range(P):
        w = want[p]
        assert got["valid"][p] == w["valid"], (B, p)
        assert got["valid_count"][p] == w["valid_count"], (B, p)
        assert got["diff"][p] == w["diff"], (B, p)
        assert got["peer_status"][p] == [STATUS.get(x, x) for x in w["status"]], (B, p)
        assert got["objects"][p] == w["object"], (B, p)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 5, 9, 64, 65])
def test_verify_epochs_peer_counts(engine, R):
    """Peer counts around the fused kernel's wave loop (4 objects staged per pass) and its limit
    (64 peers; 65 runs the chain): one partition, every peer case of _peer_objects cycled, fused
    vs chain vs oracle."""
    rng = np.random.default_rng(300 + R)
    B, E, replica = 64, 12, 3
    digests = rng.integers(0, 999999, size=B, dtype=np.uint64)
    sizes = rng.integers(0, 5000, size=B).astype(np.int32)
    _, nodes = engine.tree_from_digests(digests, B)
    pool = [o for k in range(8) for o in _peer_objects(rng, B, digests, sizes, k, E)]
    peers = [[pool[(r * 5) % len(pool)] for r in range(R)]]
    res = []
    for mode in (0, 1):
        engine.set_verify_mode(mode)
        try:
            res.append(engine.verify_epochs(B, digests, sizes, nodes, peers, replica, E))
        finally:
            engine.set_verify_mode(0)
    assert res[0] == res[1]
    w = _oracle_verify(B, digests, sizes, peers, replica, E, np.zeros(1, np.int32))[0]
    assert res[0]["valid"][0] == w["valid"] and res[0]["valid_count"][0] == w["valid_count"]
    assert res[0]["diff"][0] == w["diff"]
    assert res[0]["peer_status"][0] == [STATUS.get(x, x) for x in w["status"]]
    assert res[0]["objects"][0] == w["object"]


@pytest.mark.gpu
def test_verify_epochs_device_api_after_build(engine):
    """Device-resident chain: mde_build_async (nodes kept in HBM) -> mde_verify_epochs_async on
    peer objects already in HBM, checked against the host entry point."""
    import torch
    from mydatastore_amd.workload import make_workload
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    P, B, R = 64, 64, 3
    w = make_workload(engine, n_partitions=P, n_buckets=B, value_len=64, part_mode="mod",
                      n_keys=200_000)
    out = w.build()
    dg = out["digest"].cpu().numpy().view(np.uint64)
    sz = out["size"].cpu().numpy()
    rng = np.random.default_rng(5)
    peers = [_peer_objects(rng, B, dg[p * B:(p + 1) * B], sz[p * B:(p + 1) * B], p, 9)[:R] for p in range(P)]
    flat = [o or b"" for row in peers for o in row]
    off = np.zeros(len(flat) + 1, np.int64)
    off[1:] = np.cumsum([len(o) for o in flat])
    blob = torch.from_numpy(np.frombuffer(b"".join(flat) + b"\0", dtype=np.uint8).copy()).to(dev)
    doff = torch.from_numpy(off).to(dev)
    stride = int(engine.lib.mde_epoch_tree_object_max_bytes(B))
    o = {"valid": torch.zeros(P, dtype=torch.uint8, device=dev),
         "vc": torch.zeros(P, dtype=torch.int32, device=dev),
         "ids": torch.zeros(P * B, dtype=torch.int32, device=dev),
         "dc": torch.zeros(P, dtype=torch.int32, device=dev),
         "st": torch.zeros(P * R, dtype=torch.int32, device=dev),
         "obj": torch.zeros(P * stride, dtype=torch.uint8, device=dev),
         "olen": torch.zeros(P, dtype=torch.int32, device=dev)}
    engine.verify_epochs_async(P, B, None, 9, out["digest"], out["size"], out["nodes"], R, blob, doff, 2,
                               o["valid"], o["vc"], o["ids"], o["dc"], o["st"], o["obj"], stride, o["olen"])
    torch.cuda.synchronize()
    ref = engine.verify_epochs(B, dg, sz, out["nodes"].cpu().numpy(), peers, 2, 9)
    assert [bool(x) for x in o["valid"].cpu().tolist()] == ref["valid"]
    assert o["vc"].cpu().tolist() == ref["valid_count"]
    ids, dc = o["ids"].cpu().numpy(), o["dc"].cpu().numpy()
    assert [ids[p * B:p * B + dc[p]].tolist() for p in range(P)] == ref["diff"]
    st = o["st"].cpu().numpy()
    assert [st[p * R:(p + 1) * R].tolist() for p in range(P)] == ref["peer_status"]
    ob, ol = o["obj"].cpu().numpy(), o["olen"].cpu().numpy()
    assert [ob[p * stride:p * stride + ol[p]].tobytes() for p in range(P)] == ref["objects"]
    # and the oracle on the same trees
    want = _oracle_verify(B, dg, sz, peers, 2, 9, np.zeros(P, np.int32))
    assert [x["valid"] for x in want] == ref["valid"]
    assert [x["diff"] for x in want] == ref["diff"]


@pytest.mark.gpu
def test_verify_epochs_large_call_equals_small_calls(engine):
    """A host call too large for the packed staging (nodes alone 10 MB > 8 MiB: direct copies)
    returns exactly what the same partitions give in small packed calls (oracle-checked above)."""
    rng = np.random.default_rng(77)
    P, B, E, replica = 5000, 64, 3, 2
    digests = rng.integers(0, 999999, size=P * B, dtype=np.uint64)
    sizes = rng.integers(0, 5000, size=P * B).astype(np.int32)
    _, nodes = engine.tree_from_digests(digests, B)
    assert nodes.nbytes > 8 << 20
    peers = [_peer_objects(rng, B, digests[p * B:(p + 1) * B], sizes[p * B:(p + 1) * B], p, E)
             for p in range(P)]
    big = engine.verify_epochs(B, digests, sizes, nodes, peers, replica, E)
    NI = nodes.size // P
    for lo in range(0, P, 1000):
        hi = lo + 1000
        small = engine.verify_epochs(B, digests[lo * B:hi * B], sizes[lo * B:hi * B], nodes[lo * NI:hi * NI],
                                     peers[lo:hi], replica, E)
        for k in big:
            assert big[k][lo:hi] == small[k], (k, lo)


@pytest.mark.gpu
def test_diff_large_call_equals_small_calls(engine):
    """mde_diff over 20,000 pairs (direct copies) == the same pairs in packed calls of 1,000."""
    rng = np.random.default_rng(78)
    T, B = 20000, 64
    da = rng.integers(0, 999999, T * B).astype(np.uint64)
    db = da.copy()
    flip = rng.random(T * B) < 0.02
    db[flip] = (db[flip] + 1) % 999999
    _, na = engine.tree_from_digests(da, B)
    _, nb = engine.tree_from_digests(db, B)
    assert na.nbytes > 8 << 20
    big = engine.diff(B, da, na, B, db, nb, n_pairs=T)
    NI = na.size // T
    for lo in range(0, T, 1000):
        hi = lo + 1000
        small = engine.diff(B, da[lo * B:hi * B], na[lo * NI:hi * NI], B, db[lo * B:hi * B], nb[lo * NI:hi * NI],
                            n_pairs=1000)
        assert big[lo:hi] == small, lo


@pytest.mark.gpu
def test_verify_epochs_fuzz_fused_chain_oracle(engine):
    """Seeded fuzz of the whole decision step: 120 partitions with random B (1..70), each with
    1-6 peer objects drawn from perturbed copies, other bucket counts (shallower, same depth,
    deeper), odd-B duplicates, absent peers and byte-mutated objects. Fused launch == chain ==
    oracle on every output (valid, validCount, diffSet, peer statuses, persisted object)."""
    from tests.test_wire import _mutate
    rng = np.random.default_rng(4242)
    for trial in range(120):
        B = int(rng.integers(1, 71))
        E, replica = int(rng.integers(0, 50)), int(rng.integers(1, 4))
        digests = rng.integers(0, 999999, size=B, dtype=np.uint64)
        sizes = rng.integers(0, 3000, size=B).astype(np.int32)
        _, nodes = engine.tree_from_digests(digests, B)
        d, s = [int(x) for x in digests], [int(x) for x in sizes]
        peers = []
        for _ in range(int(rng.integers(1, 7))):
            kind = int(rng.integers(0, 6))
            if kind == 0:
                peers.append(None)
                continue
            dd, ss = list(d), list(s)
            if kind in (1, 5):  # perturb some buckets
                for b in rng.choice(B, size=int(rng.integers(1, B + 1)), replace=False):
                    dd[b] = (dd[b] + 1 + int(rng.integers(0, 999997))) % 999999
            elif kind == 2:     # another bucket count
                nb = max(1, int(rng.integers(1, 2 * B + 2)))
                dd = [int(x) for x in rng.integers(0, 999999, nb)] if nb > B else dd[:nb]
                ss = [int(x) for x in rng.integers(0, 3000, len(dd))]
            obj = wire_pb.marshal(trial, E, E + 1, dd, ss, valid=bool(rng.integers(0, 2)))
            if kind == 5:
                obj = _mutate(rng, obj)
            peers.append(obj)
        res = []
        for mode in (0, 1):
            engine.set_verify_mode(mode)
            try:
                res.append(engine.verify_epochs(B, digests, sizes, nodes, [peers], replica, E,
                                                partition=np.array([trial], np.int32)))
            finally:
                engine.set_verify_mode(0)
        assert res[0] == res[1], trial
        w = _oracle_verify(B, digests, sizes, [peers], replica, E, np.array([trial], np.int32))[0]
        g = res[0]
        assert g["valid"][0] == w["valid"] and g["valid_count"][0] == w["valid_count"], trial
        assert g["diff"][0] == w["diff"], trial
        assert g["peer_status"][0] == [STATUS.get(x, x) for x in w["status"]], trial
        assert g["objects"][0] == w["object"], trial
