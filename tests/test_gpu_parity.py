"""GPU parity: the HIP engine (through the C ABI) against the golden fixtures and the C oracle.

Bit-exact for every output (digests, sizes, items, roots, every internal node, diff id lists).
Full-size configs are checked through size-independent properties (mod-sum linearity per
partition, single-byte perturbation -> single-bucket diff, determinism, tree-of-digests).
"""
import hashlib

import numpy as np
import pytest

from oracle import oracle as O
from tests.datasets import mtr_arena, synth_arrays

pytestmark = pytest.mark.gpu


def _roots(out, P):
    return [out["root"][32 * p:32 * p + 32].tobytes().hex() for p in range(P)]


def _node_shas(out, P, B):
    ni = O.n_internal_nodes(B) * 32
    return [hashlib.sha256(out["nodes"][p * ni:(p + 1) * ni].tobytes()).hexdigest() for p in range(P)]


def test_synth_cases_host_api(engine, golden, coracle):
    for case in golden("synth_cases.json"):
        values, voff, stride, seg = synth_arrays(case, coracle)
        out = engine.build(values, seg, case["P"], case["B"], stride, voff)
        assert out["digest"].tolist() == case["digest"], case["name"]
        assert out["size"].tolist() == case["size"], case["name"]
        assert out["items"].tolist() == case["items"], case["name"]
        assert _roots(out, case["P"]) == case["root"], case["name"]
        assert _node_shas(out, case["P"], case["B"]) == case["nodes_sha256"], case["name"]


def test_synth_cases_device_api(engine, golden, coracle):
    """Device-resident path (mde_build_async) on torch-allocated HBM buffers, with a misaligned
    arena start (the kernel realigns to 16 B)."""
    import torch
    import mydatastore_amd as mde
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for case in golden("synth_cases.json"):
        values, voff, stride, seg = synth_arrays(case, coracle)
        P, B = case["P"], case["B"]
        for shift in (0, 5, 11):
            buf = torch.zeros(values.size + 32, dtype=torch.uint8, device=dev)
            buf[shift:shift + values.size] = torch.from_numpy(values).to(dev)
            dv = buf[shift:shift + values.size]
            dseg = torch.from_numpy(seg.view(np.int64)).to(dev)
            dvo = torch.from_numpy(voff.view(np.int64)).to(dev) if voff is not None else None
            rec = mde.Records(dv.data_ptr() if values.size else 0, values.size, stride, 0,
                              dvo.data_ptr() if dvo is not None else 0, case["n"], P, B,
                              dseg.data_ptr())
            o = {"digest": torch.zeros(P * B, dtype=torch.int64, device=dev),
                 "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
                 "items": torch.zeros(P, dtype=torch.int32, device=dev),
                 "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev),
                 "nodes": torch.zeros(P * O.n_internal_nodes(B) * 32, dtype=torch.uint8, device=dev)}
            to = mde.TreeOut(*(o[k].data_ptr() for k in ("digest", "size", "items", "root", "nodes")))
            engine.build_async(rec, to)
            engine.synchronize()
            out = {k: v.cpu().numpy() for k, v in o.items()}
            assert out["digest"].view(np.uint64).tolist() == case["digest"], (case["name"], shift)
            assert out["size"].tolist() == case["size"]
            assert out["items"].tolist() == case["items"]
            assert _roots(out, P) == case["root"]
            assert _node_shas(out, P, B) == case["nodes_sha256"]


@pytest.mark.parametrize("name", ["testmerkletreeraw_n100.json", "testmerkletreeraw_n10.json"])
def test_testmerkletreeraw(engine, golden, name):
    """main/merkle_tree_test.go:15-185 on the device: tagging, three builds, wire round trip,
    diffs -- every relation the reference asserts plus the absolute oracle bytes."""
    fix = golden(name)
    B = fix["n_buckets"]
    keys = [k.encode() for k, _, _ in fix["writes"]]
    bk, pt = engine.tag_keys(keys, B, 1)
    assert bk.tolist() == [fix["bucket_of"][k.decode()] for k in keys]
    assert pt.tolist() == [0] * len(keys)
    outs = {}
    for key, tr in fix["trees"].items():
        lo, hi = map(int, key.split("_"))
        vals, seg = mtr_arena(fix, lo, hi)
        out = engine.build(vals, seg, 1, B, 8)
        assert out["digest"].tolist() == tr["digests"]
        assert out["size"].tolist() == tr["sizes"]
        assert int(out["items"][0]) == tr["items"]
        assert out["root"].tobytes().hex() == tr["root"]
        assert out["nodes"].tobytes().hex() == tr["nodes"]
        # EpochTreeObjectToMerkleTree(MerkleTreeToPartitionEpochObject(tree)) keeps the root
        dec = np.array([int.from_bytes(bytes.fromhex(h), "little") for h in tr["object_buckets"]],
                       np.uint64)
        root, _ = engine.tree_from_digests(dec, len(dec))
        assert root.tobytes().hex() == tr["root"]
        outs[key] = out
    t1, t2, t3 = outs["0_3"], outs["1_3"], outs["2_3"]
    assert t1["root"].tobytes() == t2["root"].tobytes() != t3["root"].tobytes()

    def d(a, b):
        return engine.diff(B, a["digest"], a["nodes"], B, b["digest"], b["nodes"])[0]

    assert d(t1, t2) == fix["diffs"]["t1_t2"] == []
    assert d(t2, t1) == fix["diffs"]["t2_t1"] == []
    assert d(t1, t3) == fix["diffs"]["t1_t3"] and len(d(t1, t3)) > 0
    assert d(t3, t1) == fix["diffs"]["t3_t1"]


def test_diff_cases(engine, golden):
    import mydatastore_amd as mde
    for c in golden("diff_cases.json"):
        da, db = np.array(c["d1"], np.uint64), np.array(c["d2"], np.uint64)
        ra, na = engine.tree_from_digests(da, c["b1"])
        rb, nb = engine.tree_from_digests(db, c["b2"])
        got = engine.diff(c["b1"], da, na, c["b2"], db, nb)[0]
        got2 = engine.diff_digests(c["b1"], da, c["b2"], db)[0]
        assert got == got2, c["name"]
        if "error" in c:
            assert got == mde.MDE_E_TREE, c["name"]
        else:
            assert got == c["ids"], c["name"]


def test_diff_batched(engine, coracle):
    """Many pairs per launch (the C5 compare step), random perturbations, B = 64 and 30."""
    rng = np.random.default_rng(11)
    for B in (64, 30, 1000):
        P = 40
        da = rng.integers(0, O.HASH_MOD, P * B).astype(np.uint64)
        db = da.copy()
        for p in range(P):
            k = rng.integers(0, 4)
            idx = rng.choice(B, size=k, replace=False)
            db[p * B + idx] = (db[p * B + idx] + 1) % O.HASH_MOD
        _, na = engine.tree_from_digests(da, B)
        _, nb = engine.tree_from_digests(db, B)
        got = engine.diff(B, da, na, B, db, nb, n_pairs=P)
        for p in range(P):
            assert got[p] == coracle.diff(da[p * B:(p + 1) * B], db[p * B:(p + 1) * B]), (B, p)


def test_tree_from_digests_matches_oracle(engine, coracle):
    rng = np.random.default_rng(3)
    for B in (1, 2, 3, 5, 30, 64, 100, 1000, 4096, 4097, 10001):
        T = 3
        d = rng.integers(0, 2**63, T * B, dtype=np.int64).astype(np.uint64)  # any int64 on the wire
        root, nodes = engine.tree_from_digests(d, B)
        ni = O.n_internal_nodes(B) * 32
        for t in range(T):
            r, n = coracle.tree(d[t * B:(t + 1) * B], B)
            assert root[32 * t:32 * t + 32].tobytes() == r, B
            assert nodes[t * ni:(t + 1) * ni].tobytes() == n, B
    # >= 512 wide trees: the tree kernel's pair shape (two trees per workgroup), odd tree counts
    for B, T in ((257, 515), (1000, 513)):
        d = rng.integers(0, 2**63, T * B, dtype=np.int64).astype(np.uint64)
        root, nodes = engine.tree_from_digests(d, B)
        ni = O.n_internal_nodes(B) * 32
        for t in range(T):
            r, n = coracle.tree(d[t * B:(t + 1) * B], B)
            assert root[32 * t:32 * t + 32].tobytes() == r, (B, t)
            assert nodes[t * ni:(t + 1) * ni].tobytes() == n, (B, t)


def test_tag_kernels(engine, golden, coracle):
    import torch
    k = golden("kat_hash.json")
    keys = [bytes.fromhex(r[0]) for r in k["key_tags"]]
    b64, p15 = engine.tag_keys(keys, 64, 15)
    b1000, p1024 = engine.tag_keys(keys, 1000, 1024)
    assert b64.tolist() == [r[1] for r in k["key_tags"]]
    assert b1000.tolist() == [r[2] for r in k["key_tags"]]
    assert p15.tolist() == [r[3] for r in k["key_tags"]]
    assert p1024.tolist() == [r[4] for r in k["key_tags"]]
    # variable-length keys exercising multi-block SHA and every XXH64 branch
    keys = [bytes.fromhex(m) for m, _ in k["xxh64"]]
    bk, pt = engine.tag_keys(keys, 1 << 31, 2**32 - 1)
    for key, b, p in zip(keys, bk, pt):
        assert b == O.get_key_bucket(key, 1 << 31)
        assert p == O.xxh64(key) % (2**32 - 1)
    # synthetic tag + value kernels == C oracle
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    gids = np.arange(5000, dtype=np.uint64) * np.uint64(7919) + np.uint64(3)
    dg = torch.from_numpy(gids.view(np.int64)).to(dev)
    for mode, P, kpp in ((0, 7, 800), (1, 1024, 0), (2, 15, 0)):
        part = torch.zeros(5000, dtype=torch.int32, device=dev)
        bkt = torch.zeros(5000, dtype=torch.int32, device=dev)
        engine.synth_tags_async(dg, 5000, P, 64, mode, max(kpp, 1) if mode == 0 else 0, part, bkt)
        engine.synchronize()
        ep, eb = coracle.synth_tags(gids, P, 64, mode, max(kpp, 1))
        assert part.cpu().numpy().view(np.uint32).tolist() == ep.tolist()
        assert bkt.cpu().numpy().view(np.uint32).tolist() == eb.tolist()
    for vl in (8, 13, 64, 1024):
        dst = torch.zeros(5000 * vl, dtype=torch.uint8, device=dev)
        engine.synth_values_async(dst, dg, 5000, vl, O.SYNTH_SEED)
        engine.synchronize()
        assert np.array_equal(dst.cpu().numpy(), coracle.synth_values(gids, vl, O.SYNTH_SEED))


def test_edge_cases(engine, coracle):
    rng = np.random.default_rng(5)
    # zero records, all buckets empty
    out = engine.build(np.zeros(0, np.uint8), np.zeros(3 * 8 + 1, np.uint64), 3, 8, 16)
    exp = coracle.build(np.zeros(0, np.uint8), np.zeros(3 * 8 + 1, np.uint64), 3, 8, 16)
    assert out["root"].tobytes() == exp["root"].tobytes() and out["digest"].sum() == 0
    # one huge bucket spanning many wave ranges, tiny neighbours, odd stride
    for stride, counts in ((7, [1, 200000, 0, 3]), (1, [5, 0, 0, 9, 1]), (1024, [3000, 1, 0, 2999])):
        B = len(counts)
        seg = np.zeros(B + 1, np.uint64)
        np.cumsum(counts, out=seg[1:])
        vals = rng.integers(0, 256, int(seg[-1]) * stride, dtype=np.uint8)
        out = engine.build(vals, seg, 1, B, stride)
        exp = coracle.build(vals, seg, 1, B, stride)
        for k in ("digest", "size", "items", "root", "nodes"):
            assert np.array_equal(out[k], exp[k]), (stride, k)
    # values of 0xff everywhere: sums close to the u32 lane limits stay exact
    vals = np.full(1 << 24, 255, np.uint8)
    seg = np.array([0, 1 << 16, 1 << 20], np.uint64)  # record indices (16-byte records)
    out = engine.build(vals, seg, 1, 2, 16)
    assert out["digest"].tolist() == [((1 << 20) * 255) % O.HASH_MOD,
                                      ((1 << 24) - (1 << 20)) * 255 % O.HASH_MOD]
    # malformed input is rejected on the host API (never reaches a kernel)
    import mydatastore_amd as mde
    with pytest.raises(mde.MdeError) as e:
        engine.build(vals, np.array([0, 1 << 16, 1 << 24], np.uint64), 1, 2, 16)
    assert e.value.code == mde.MDE_E_INVAL
    with pytest.raises(mde.MdeError):
        engine.build(vals, np.array([0, 1 << 17, 1 << 16], np.uint64), 1, 2, 16)
    # records before seg_rec[0] are not part of any bucket
    vals = rng.integers(0, 256, 64 * 10, dtype=np.uint8)
    seg = np.array([2, 5, 9], np.uint64)
    out = engine.build(vals, seg, 1, 2, 64)
    exp = coracle.build(vals, seg, 1, 2, 64)
    assert out["digest"].tolist() == exp["digest"].tolist()


def test_many_tiny_buckets(engine, coracle):
    """Production-shaped tiny values (8-byte LE timestamps), B = 1000, sparse partitions."""
    rng = np.random.default_rng(9)
    P, B = 37, 1000
    counts = rng.integers(0, 4, P * B) * (rng.random(P * B) < 0.4)
    seg = np.zeros(P * B + 1, np.uint64)
    np.cumsum(counts, out=seg[1:])
    vals = rng.integers(0, 2**40, int(seg[-1]), dtype=np.int64).view(np.uint8)
    out = engine.build(vals, seg, P, B, 8)
    exp = coracle.build(vals, seg, P, B, 8)
    for k in ("digest", "size", "items", "root", "nodes"):
        assert np.array_equal(out[k], exp[k]), k


def test_long_wave_ranges_stay_exact():
    """Arenas large enough that each streaming wave owns tens of MiB (here 20 GiB of 0xff over
    the 1,024 waves of a 1-workgroup-per-CU grid, 20 MiB per wave, C3 gives 32 MiB): the u32 lane
    accumulators stay exact and bucket boundaries at arbitrary records inside long ranges are
    honoured, in the standalone build and in the fused pipelined step."""
    import torch
    import mydatastore_amd as mde
    dev = torch.device("cuda:0")
    eng = mde.Engine(0)
    try:
        eng.set_tuning(digest_blocks_per_cu=1)
        eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        V = 16
        n = (20 << 30) // V + 3
        vals = torch.full((n * V,), 255, dtype=torch.uint8, device=dev)
        P, B = 2, 2
        seg = np.array([0, 1_234_567, 700_000_001, 700_000_002, n], np.uint64)
        dseg = torch.from_numpy(seg.view(np.int64)).to(dev)
        rec = mde.Records(vals.data_ptr(), n * V, V, mde.LAYOUT_SORTED, 0, n, P, B, dseg.data_ptr())
        cnt = np.diff(seg)
        exp = [int(c) * V * 255 % O.HASH_MOD for c in cnt]
        sets = []
        for _ in range(3):
            o = {"digest": torch.full((P * B,), -1, dtype=torch.int64, device=dev),
                 "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
                 "items": torch.zeros(P, dtype=torch.int32, device=dev),
                 "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev),
                 "nodes": torch.zeros(P * O.n_internal_nodes(B) * 32, dtype=torch.uint8, device=dev)}
            sets.append((o, mde.TreeOut(*(o[k].data_ptr() for k in ("digest", "size", "items", "root", "nodes")))))
        eng.build_async(rec, sets[0][1])
        eng.build_pipelined_async(rec, sets[1][1])
        eng.build_pipelined_async(rec, sets[2][1])
        eng.build_pipeline_drain_async()
        eng.synchronize()
        for i, (o, _) in enumerate(sets):
            assert o["digest"].cpu().numpy().view(np.uint64).tolist() == exp, i
            assert o["size"].cpu().numpy().tolist() == [int(c) for c in cnt], i
        del vals
    finally:
        eng.close()


def test_full_size_properties(engine):
    """BASELINE config 2 shape (256 partitions x 100k keys x 256 B, B = 64) generated on device:
    per-partition mod-sum linearity, sizes, roots == tree(digests), exact recomputation of
    sampled buckets, single-byte perturbation -> exactly one differing bucket, determinism."""
    import torch
    from mydatastore_amd.workload import make_workload
    w = make_workload(engine, n_partitions=256, keys_per_partition=100_000, value_len=256,
                      n_buckets=64, part_mode="block")
    P, B = 256, 64
    out1 = w.build()
    out2 = w.build()
    for k in out1:
        assert torch.equal(out1[k], out2[k]), k
    digest = out1["digest"].cpu().numpy().view(np.uint64)
    seg = w.seg_rec.cpu().numpy().view(np.uint64)
    assert out1["size"].cpu().numpy().tolist() == np.diff(seg).astype(np.int32).tolist()
    assert int(out1["items"].sum()) == P * 100_000
    # per-partition sum of values (torch on device) mod m == sum of digests mod m
    vals = w.values.view(torch.uint8)
    V = 256
    for p in list(range(0, P, 17)) + [P - 1]:
        lo, hi = int(seg[p * B]) * V, int(seg[(p + 1) * B]) * V
        tot = int(vals[lo:hi].to(torch.int64).sum().item())
        assert tot % O.HASH_MOD == int(digest[p * B:(p + 1) * B].sum()) % O.HASH_MOD
        # sampled exact buckets
        b = (p * 7) % B
        s0, s1 = int(seg[p * B + b]) * V, int(seg[p * B + b + 1]) * V
        assert int(vals[s0:s1].to(torch.int64).sum().item()) % O.HASH_MOD == int(digest[p * B + b])
    roots = out1["root"].cpu().numpy()
    for p in range(0, P, 31):
        lv = O.tree_levels_from_digests([int(x) for x in digest[p * B:(p + 1) * B]])
        assert roots[32 * p:32 * p + 32].tobytes() == lv[-1][0]
    # perturb one byte in bucket (p*37) % 64 of every 16th partition: diff == [that bucket]
    touched = {}
    for p in range(0, P, 16):
        b = (p * 37) % B
        r = int(seg[p * B + b])
        if int(seg[p * B + b + 1]) > r:
            vals[r * V] = (vals[r * V].to(torch.int32) + 1).remainder(256).to(torch.uint8)
            touched[p] = b
    out3 = w.build()
    ids = w.diff(out1, out3)
    for p in range(P):
        assert ids[p] == ([touched[p]] if p in touched else []), p


def _extract_case(engine, values, voff, stride, seg, P, B, ids, stride_ids, counts):
    vo = voff if voff is not None else np.arange(len(values) // stride + 1, dtype=np.uint64) * np.uint64(stride)
    exp = O.extract_from_arena(values, vo, seg, P, B, ids, stride_ids, counts)
    got = engine.extract(values, seg, P, B, ids, stride_ids, counts, stride, voff)
    for g, e, name in zip(got, exp, ("part_off", "rec", "values", "value_off")):
        assert np.array_equal(np.asarray(g), e), name


def test_extract_matches_oracle(engine, golden, coracle):
    """Range extract over random (duplicated, unordered, out-of-range) bucket lists."""
    rng = np.random.default_rng(21)
    for case in golden("synth_cases.json"):
        P, B = case["P"], case["B"]
        if B > 65536:
            continue
        values, voff, stride, seg = synth_arrays(case, coracle)
        cap = 8
        ids = rng.integers(-2, B + 2, P * cap).astype(np.int32)
        counts = rng.integers(-1, cap + 1, P).astype(np.int32)
        _extract_case(engine, values, voff, stride, seg, P, B, ids, cap, counts)
        # every bucket requested (StreamBuckets with an empty list = all buckets)
        ids = np.tile(np.arange(B, dtype=np.int32), P)
        _extract_case(engine, values, voff, stride, seg, P, B, ids, B, np.full(P, B, np.int32))


def test_extract_streambuckets_scenario(engine, golden):
    """TestStreamBucketsTask-style (main/manager_test.go:117-211): the diff set of t1 vs t3 of the
    TestMerkleTreeRaw scenario streams exactly the records the reference's range scans yield,
    and their LE64 values decode to the written timestamps."""
    fix = golden("testmerkletreeraw_n100.json")
    B = fix["n_buckets"]
    vals, seg = mtr_arena(fix, 0, 3)
    diff = fix["diffs"]["t1_t3"]
    part_off, rec, vbytes, voff = engine.extract(vals, seg, 1, B, np.array(diff, np.int32), len(diff),
                                                 np.array([len(diff)], np.int32), 8)
    want = sorted((fix["bucket_of"][k], f"{e:010d}", k, ts) for k, e, ts in fix["writes"]
                  if fix["bucket_of"][k] in set(diff))
    assert int(part_off[-1]) == len(want)
    assert vbytes.view("<i8").tolist() == [w[3] for w in want]
    # all buckets, epochs [0,3): 2N records (main/manager_test.go:210)
    pa, _, _, _ = engine.extract(vals, seg, 1, B, np.arange(B, dtype=np.int32), B,
                                 np.array([B], np.int32), 8, want_values=False)
    assert int(pa[-1]) == 2 * fix["n"]


def _stream_case(engine, values, voff, stride, seg, P, B, ids, stride_ids, counts):
    vo = voff if voff is not None else np.arange(len(values) // stride + 1, dtype=np.uint64) * np.uint64(stride)
    exp = O.stream_buckets_from_arena(values, vo, seg, P, B, ids, stride_ids, counts)
    got = engine.stream_buckets(values, seg, P, B, ids, stride_ids, counts, stride, voff)
    for g, e, name in zip(got, exp, ("part_off", "rec", "values", "value_off")):
        assert np.array_equal(np.asarray(g), e), name
    return exp


def test_stream_buckets_request_order_matches_oracle(engine, golden, coracle):
    """mde_stream_buckets: StreamBucketsTask's list contract (main/manager.go:447-485) -- the ids
    walked in the order given, repeats streamed again, out-of-range ids streaming nothing,
    counts == 0 meaning every bucket, counts < 0 nothing -- against the oracle's restatement on
    random unordered lists with repeats, over every synthetic fixture shape."""
    rng = np.random.default_rng(33)
    for case in golden("synth_cases.json"):
        P, B = case["P"], case["B"]
        if B > 65536:
            continue
        values, voff, stride, seg = synth_arrays(case, coracle)
        cap = 12
        ids = rng.integers(-2, B + 2, P * cap).astype(np.int32)
        ids[1::3] = ids[0::3][:len(ids[1::3])]  # plenty of repeats
        counts = rng.integers(-1, cap + 1, P).astype(np.int32)
        _stream_case(engine, values, voff, stride, seg, P, B, ids, cap, counts)
        # the task's empty list: every bucket, ascending
        exp = _stream_case(engine, values, voff, stride, seg, P, B, np.zeros(P, np.int32), 1,
                           np.zeros(P, np.int32))
        assert int(exp[0][-1]) == int(seg[-1]) - int(seg[0])


def test_stream_buckets_repeats_and_order(engine, golden):
    """A list with repeats and out-of-range ids on the TestMerkleTreeRaw N=100 arena (B = 30):
    b1's records, bm's, b0's, then b1's again, in that order; 99, 1000 and -1 stream nothing. The
    deduplicated mde_extract on the same list returns each bucket once, ascending."""
    fix = golden("testmerkletreeraw_n100.json")
    B = fix["n_buckets"]
    vals, seg = mtr_arena(fix, 0, 3)
    nonempty = [b for b in range(B) if seg[b + 1] > seg[b]]
    b0, bm, b1 = nonempty[0], nonempty[len(nonempty) // 2], nonempty[-1]
    req = np.array([b1, 99, bm, -1, b0, b1, 1000], np.int32)
    part_off, rec, vbytes, voff = engine.stream_buckets(vals, seg, 1, B, req, len(req),
                                                        np.array([len(req)], np.int32), 8)
    runs = [list(range(int(seg[b]), int(seg[b + 1]))) for b in (b1, bm, b0, b1)]
    assert rec.tolist() == [r for run in runs for r in run]
    assert vbytes.tobytes() == b"".join(vals[r * 8:(r + 1) * 8].tobytes() for run in runs for r in run)
    assert voff.tolist() == list(range(0, 8 * len(rec) + 1, 8))
    _, drec, _, _ = engine.extract(vals, seg, 1, B, req, len(req), np.array([len(req)], np.int32), 8)
    assert drec.tolist() == [r for b in sorted({b0, bm, b1}) for r in range(int(seg[b]), int(seg[b + 1]))]


def test_stream_buckets_rejects_layout_b(engine):
    import ctypes as C
    import mydatastore_amd as mde
    vals = np.zeros(64, np.uint8)
    tag = np.zeros(8, np.uint16)
    prec = np.array([0, 8], np.uint64)
    rec = mde.Records(vals.ctypes.data, vals.nbytes, 8, mde.LAYOUT_TAGGED, 0, 8, 1, 4, 0,
                      tag.ctypes.data, prec.ctypes.data)
    ids = np.array([0], np.int32)
    cnt = np.array([1], np.int32)
    po = np.zeros(2, np.uint64)
    out = np.zeros(8, np.uint64)
    rc = engine.lib.mde_stream_buckets(engine.ctx, C.byref(rec), ids.ctypes.data, 1, cnt.ctypes.data,
                                       po.ctypes.data, out.ctypes.data, 8, None, None, 0)
    assert rc == mde.MDE_E_INVAL


def test_extract_capacity_error(engine):
    import ctypes as C
    import mydatastore_amd as mde
    vals = np.arange(64 * 4, dtype=np.uint8)
    seg = np.array([0, 2, 4], np.uint64)
    rec = mde.Records(vals.ctypes.data, vals.nbytes, 64, 0, 0, 4, 1, 2, seg.ctypes.data)
    ids = np.array([0, 1], np.int32)
    cnt = np.array([2], np.int32)
    po = np.zeros(2, np.uint64)
    out = np.zeros(2, np.uint64)
    rc = engine.lib.mde_extract(engine.ctx, C.byref(rec), ids.ctypes.data, 2, cnt.ctypes.data,
                                po.ctypes.data, out.ctypes.data, 2, None, None, 0)
    assert rc == mde.MDE_E_CAPACITY and int(po[-1]) == 4


def test_build_streamed_matches_oracle(engine, golden, coracle):
    """Host ingest path: chunked two-slot ring (tiny chunks force many chunks and odd alignments)."""
    for case in golden("synth_cases.json"):
        values, voff, stride, seg = synth_arrays(case, coracle)
        P, B = case["P"], case["B"]
        for chunk in (1, 777, 0):
            out = engine.build_streamed(values, seg, P, B, stride, voff, chunk_bytes=chunk)
            assert out["digest"].tolist() == case["digest"], (case["name"], chunk)
            assert out["size"].tolist() == case["size"]
            assert out["items"].tolist() == case["items"]
            assert _roots(out, P) == case["root"]
            assert _node_shas(out, P, B) == case["nodes_sha256"]


def test_build_streamed_layout_b(engine, golden, coracle):
    """Host ingest of layout B (write order + tags) through the same ring, chunk sizes that split
    the arena at every partition."""
    from tests.datasets import MODES
    for case in golden("synth_cases.json"):
        if case["var_len"]:
            continue
        n, P, B, V = case["n"], case["P"], case["B"], case["value_len"]
        gids = np.arange(n, dtype=np.uint64)
        part, bk = coracle.synth_tags(gids, P, B, MODES[case["part_mode"]], case["keys_per_partition"])
        order = np.argsort(part, kind="stable")
        part_rec = np.zeros(P + 1, np.uint64)
        np.cumsum(np.bincount(part, minlength=P), out=part_rec[1:])
        values = coracle.synth_values(gids[order], V, case["seed"])
        for chunk in (1, 4099, 0):
            out = engine.build_streamed(values, None, P, B, V, chunk_bytes=chunk, part_rec=part_rec,
                                        bucket_tag=bk[order].astype(np.uint16))
            assert out["digest"].tolist() == case["digest"], (case["name"], chunk)
            assert out["size"].tolist() == case["size"], (case["name"], chunk)
            assert out["items"].tolist() == case["items"], (case["name"], chunk)
            assert _roots(out, P) == case["root"], (case["name"], chunk)
            assert _node_shas(out, P, B) == case["nodes_sha256"], (case["name"], chunk)


def test_layout_b_matches_fixtures(engine, golden, coracle):
    """Layout B (arrival order within a partition + bucket tags): the engine bins records into
    buckets itself; same record sets as the golden builds, identical outputs."""
    from tests.datasets import MODES
    for case in golden("synth_cases.json"):
        if case["var_len"] or case["B"] > 65536:
            continue
        n, P, B, V = case["n"], case["P"], case["B"], case["value_len"]
        gids = np.arange(n, dtype=np.uint64)
        part, bk = coracle.synth_tags(gids, P, B, MODES[case["part_mode"]], case["keys_per_partition"])
        order = np.argsort(part, kind="stable")          # grouped by partition, gid order inside
        part_rec = np.zeros(P + 1, np.uint64)
        np.cumsum(np.bincount(part, minlength=P), out=part_rec[1:])
        values = coracle.synth_values(gids[order], V, case["seed"])
        out = engine.build_tagged(values, part_rec, bk[order].astype(np.uint16), P, B, V)
        assert out["digest"].tolist() == case["digest"], case["name"]
        assert out["size"].tolist() == case["size"], case["name"]
        assert out["items"].tolist() == case["items"], case["name"]
        assert _roots(out, P) == case["root"], case["name"]
        assert _node_shas(out, P, B) == case["nodes_sha256"], case["name"]


def test_layout_b_tiny_and_odd_strides(engine, coracle):
    """Records of 1..37 bytes (several per 16-byte vector), partitions with empty gaps."""
    rng = np.random.default_rng(41)
    for V in (1, 3, 7, 8, 13, 16, 24, 37, 100, 1024, 1031):
        P, B = 5, 16
        counts = rng.integers(0, 400, P)
        counts[2] = 0
        part_rec = np.zeros(P + 1, np.uint64)
        np.cumsum(counts, out=part_rec[1:])
        n = int(part_rec[-1])
        tags = rng.integers(0, B, n).astype(np.uint16)
        values = rng.integers(0, 256, n * V, dtype=np.uint8)
        out = engine.build_tagged(values, part_rec, tags, P, B, V)
        # oracle: layout A of the same records (stable sort by (partition, tag))
        part = np.repeat(np.arange(P), counts)
        order = np.lexsort((tags, part))
        seg = np.zeros(P * B + 1, np.uint64)
        np.cumsum(np.bincount(part * B + tags.astype(np.int64), minlength=P * B), out=seg[1:])
        vals_a = values.reshape(n, V)[order].reshape(-1) if n else values
        exp = coracle.build(vals_a, seg, P, B, V)
        for k in ("digest", "size", "items", "root", "nodes"):
            assert np.array_equal(out[k], exp[k]), (V, k)


def test_layout_b_full_size_equals_layout_a(engine):
    """C4 shard (128 partitions x 1 KiB values, 1.28 GB): layout B over arrival order gives the
    same digests/sizes/roots as layout A over the sorted order."""
    import torch
    from mydatastore_amd.workload import make_workload
    kw = dict(n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod", n_keys=10_000_000,
              rank=3, world=8)
    wa = make_workload(engine, **kw)
    oa = wa.build()
    del wa
    wb = make_workload(engine, layout="b", **kw)
    ob = wb.build()
    for k in ("digest", "size", "items", "root", "nodes"):
        assert torch.equal(oa[k], ob[k]), k


def test_extract_layout_b(engine):
    """Range extract over layout B (write order + tags): the records of the requested buckets
    (duplicates / out-of-range ids ignored), per partition in arrival order, values included."""
    rng = np.random.default_rng(77)
    for V, B in ((8, 30), (64, 64), (1024, 64), (37, 1000), (16, 7)):
        P = 6
        counts = rng.integers(0, 700, P)
        counts[3] = 0
        part_rec = np.zeros(P + 1, np.uint64)
        np.cumsum(counts, out=part_rec[1:])
        n = int(part_rec[-1])
        tags = rng.integers(0, B, n).astype(np.uint16)
        values = rng.integers(0, 256, n * V, dtype=np.uint8)
        cap = 6
        ids = rng.integers(-2, B + 2, P * cap).astype(np.int32)
        req = rng.integers(-1, cap + 1, P).astype(np.int32)
        part_off, rec, vbytes, voff = engine.extract(values, None, P, B, ids, cap, req, value_stride=V,
                                                     part_rec=part_rec, bucket_tag=tags)
        want, wpo = [], [0]
        for p in range(P):
            sel = {int(b) for b in ids[p * cap:p * cap + max(int(req[p]), 0)] if 0 <= b < B}
            want += [r for r in range(int(part_rec[p]), int(part_rec[p + 1])) if int(tags[r]) in sel]
            wpo.append(len(want))
        assert part_off.tolist() == wpo, (V, B)
        assert rec.tolist() == want, (V, B)
        wv = values.reshape(max(n, 1), -1)[want].reshape(-1) if want else np.zeros(0, np.uint8)
        assert np.array_equal(vbytes, wv), (V, B)
        assert voff.tolist() == [i * V for i in range(len(want) + 1)], (V, B)


def test_abi_error_paths(engine):
    """Bad arguments come back as MDE_E_* codes with a message -- never a crash or a fault."""
    import ctypes as C
    import mydatastore_amd as mde
    lib, ctx = engine.lib, engine.ctx
    vals = np.zeros(1024, np.uint8)
    seg = np.array([0, 4, 2, 8], np.uint64)  # not nondecreasing
    digest = np.zeros(3, np.uint64)
    size = np.zeros(3, np.int32)
    items = np.zeros(1, np.int32)
    root = np.zeros(32, np.uint8)
    out = mde.TreeOut(digest.ctypes.data, size.ctypes.data, items.ctypes.data, root.ctypes.data, 0)

    def rc_of(rec):
        return lib.mde_build(ctx, C.byref(rec), C.byref(out))

    assert lib.mde_build(ctx, None, C.byref(out)) == mde.MDE_E_INVAL
    assert rc_of(mde.Records(vals.ctypes.data, vals.nbytes, 64, 0, 0, 8, 1, 3, seg.ctypes.data)) == mde.MDE_E_INVAL
    assert b"nondecreasing" in lib.mde_last_error(ctx)
    good = np.array([0, 4, 6, 8], np.uint64)
    assert rc_of(mde.Records(vals.ctypes.data, vals.nbytes, 64, 7, 0, 8, 1, 3, good.ctypes.data)) == mde.MDE_E_INVAL
    # stride * records beyond the arena
    assert rc_of(mde.Records(vals.ctypes.data, vals.nbytes, 256, 0, 0, 8, 1, 3, good.ctypes.data)) == mde.MDE_E_INVAL
    # layout B: a tag out of range, a missing part_rec
    tags = np.array([0, 1, 5, 2], np.uint16)
    pr = np.array([0, 4], np.uint64)
    assert rc_of(mde.Records(vals.ctypes.data, vals.nbytes, 64, 1, 0, 4, 1, 3, 0, tags.ctypes.data,
                             pr.ctypes.data)) == mde.MDE_E_INVAL
    assert rc_of(mde.Records(vals.ctypes.data, vals.nbytes, 64, 1, 0, 4, 1, 3, 0, tags.ctypes.data, 0)) == mde.MDE_E_INVAL
    # capacities
    ids = np.zeros(4, np.int32)
    cnt = np.zeros(1, np.int32)
    d64 = np.zeros(64, np.uint64)
    n64 = np.zeros(mde.tree_internal_nodes(64) * 32, np.uint8)
    assert lib.mde_diff(ctx, 1, 64, d64.ctypes.data, n64.ctypes.data, 64, d64.ctypes.data, n64.ctypes.data,
                        ids.ctypes.data, 4, cnt.ctypes.data) == mde.MDE_E_CAPACITY
    o = np.zeros(16, np.uint8)
    ln = np.zeros(1, np.uint32)
    s64 = np.zeros(64, np.int32)
    assert lib.mde_encode_epoch_tree_objects(ctx, 1, 64, None, 0, 1, d64.ctypes.data, s64.ctypes.data, None, None,
                                             o.ctypes.data, 16, ln.ctypes.data) == mde.MDE_E_CAPACITY
    assert lib.mde_tree_from_digests(ctx, 1, 0, d64.ctypes.data, root.ctypes.data, None) == mde.MDE_E_INVAL
    v = np.zeros(1, np.uint8)
    assert lib.mde_verify_epochs(ctx, 1, 0, None, 0, d64.ctypes.data, s64.ctypes.data, n64.ctypes.data, 0, None,
                                 None, 1, v.ctypes.data, cnt.ctypes.data, ids.ctypes.data, cnt.ctypes.data, None,
                                 None, 0, None) == mde.MDE_E_INVAL
    # device groups: a device that does not exist
    devs = (C.c_int * 2)(0, 99)
    h = C.c_void_p()
    assert lib.mde_group_create(devs, 2, C.byref(h)) == mde.MDE_E_INVAL and not h.value
    # the engine still works after every rejected call
    good_out = engine.build(np.arange(256, dtype=np.uint8), np.array([0, 2, 4], np.uint64), 1, 2, 64)
    assert good_out["size"].tolist() == [2, 2]
