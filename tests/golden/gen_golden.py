"""Generate the committed golden fixtures in tests/golden/ from the CPU oracle (oracle/oracle.py).

    python tests/golden/gen_golden.py

Inputs are synthetic and fully determined by the parameters stored in each fixture (seeded
splitmix64 values, "k%016x" keys) or by the reference's own test scenarios
(main/merkle_tree_test.go:15-185, main/indexs_test.go, storage/index_test.go). Expected outputs
come from the oracle, whose parity status is documented in oracle/oracle.py.
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
from oracle import oracle as O  # noqa: E402
from oracle import wire_pb  # noqa: E402


def _hex(b: bytes) -> str:
    return bytes(b).hex()


def testmerkletreeraw(n: int, n_buckets: int = 30) -> dict:
    """main/merkle_tree_test.go:15-185 with N = n (100, or 10 under -test.short)."""
    m = O.Manager(partition_count=1, partition_buckets=n_buckets)
    ts = 0
    writes = []
    for i in range(n):  # epoch 1
        ts += 1
        m.set_value(f"key{i}", f"val{i}", 1, ts)
        writes.append([f"key{i}", 1, ts])
    for i in range(n):  # epoch 2
        ts += 1
        m.set_value(f"keyz{i}", f"valz{i}", 2, ts)
        writes.append([f"keyz{i}", 2, ts])
    trees = {}
    for lo, hi in ((0, 3), (1, 3), (2, 3)):
        t = m.raw_partition_merkle_tree(0, lo, hi)
        obj = O.merkle_tree_to_partition_epoch_object(t, 0, lo, hi)
        trees[f"{lo}_{hi}"] = {
            "digests": [leaf.c.hasher.hash() for leaf in t.leafs[:n_buckets]],
            "sizes": [leaf.c.size for leaf in t.leafs[:n_buckets]],
            "items": obj.items,
            "root": _hex(t.merkle_root()),
            "nodes": _hex(O.internal_nodes_blob([leaf.c.hasher.hash() for leaf in t.leafs[:n_buckets]])),
            "object_buckets": [_hex(b) for b in obj.buckets],
            # proto.Marshal(obj) (main/manager.go:1045) via the protobuf runtime
            "wire": _hex(wire_pb.epoch_tree_object_class()(
                partition=obj.partition, lower_epoch=obj.lower_epoch, upper_epoch=obj.upper_epoch,
                buckets=obj.buckets, buckets_size=obj.buckets_size, valid=obj.valid,
                items=obj.items).SerializeToString()),
        }
    t1, t2, t3 = (m.raw_partition_merkle_tree(0, lo, 3) for lo in (0, 1, 2))
    st1 = O.epoch_tree_object_to_merkle_tree(O.merkle_tree_to_partition_epoch_object(t1, 0, 0, 3))
    st3 = O.epoch_tree_object_to_merkle_tree(O.merkle_tree_to_partition_epoch_object(t3, 0, 2, 3))
    diffs = {
        "t1_t2": O.different_merkle_tree_buckets(t1, t2),
        "t2_t1": O.different_merkle_tree_buckets(t2, t1),
        "t1_t3": O.different_merkle_tree_buckets(t1, t3),
        "t3_t1": O.different_merkle_tree_buckets(t3, t1),
        "t1_st1": O.different_merkle_tree_buckets(t1, st1),
        "t1_st3": O.different_merkle_tree_buckets(t1, st3),
    }
    tags = {k: O.get_key_bucket(k.encode(), n_buckets) for k, _, _ in writes}
    return {"n": n, "n_buckets": n_buckets, "writes": writes, "bucket_of": tags, "trees": trees,
            "diffs": diffs}


def kat_index() -> dict:
    """Pinned by the reference's tests (main/indexs_test.go:18,32; storage/index_test.go:19,30)."""
    return {
        "epoch_index": [[1, 2, 3, "zz", "epoch_1_2_0000000003_zz"]],
        "epoch_tree_index": [[1, 2, "epochtree_1_0000000002"]],
        "generic": [
            ["test", ["part1", "bucket1", ["1", 4], "mykey"], "test_part1_bucket1_0001_mykey"],
            ["zzz", ["part1", "bucket1", ["100", 4], "mykey"], "zzz_part1_bucket1_0100_mykey"],
        ],
        "parse": [["epoch_1_2_0000000003_zz", 1, 2, 3, "zz"]],
    }


def kat_hash() -> dict:
    msgs = [b"", b"abc", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
            b"a" * 55, b"a" * 56, b"a" * 64, b"a" * 119, b"a" * 200]
    lengths = list(range(0, 70)) + [100, 255, 1000]
    xx_msgs = [bytes((i * 7 + 3) & 0xFF for i in range(n)) for n in lengths]
    return {
        # FIPS 180-4 examples ("", "abc", 448-bit) are published vectors; the rest exercise padding.
        "sha256": [[_hex(m), hashlib.sha256(m).hexdigest()] for m in msgs],
        # XXH64 published: XXH64("",0)=ef46db3751d8e999, XXH64("abc",0)=44bc2cf5ad770999.
        "xxh64_published": [["", "ef46db3751d8e999"], [_hex(b"abc"), "44bc2cf5ad770999"]],
        "xxh64": [[_hex(m), "%016x" % O.xxh64(m)] for m in xx_msgs],
        "key_tags": [[_hex(O.synth_key(g)), O.get_key_bucket(O.synth_key(g), 64),
                      O.get_key_bucket(O.synth_key(g), 1000), O.find_partition_id(O.synth_key(g), 15),
                      O.find_partition_id(O.synth_key(g), 1024)] for g in range(0, 4000, 37)],
        "splitmix_words": [[g, w, "%016x" % int(O.synth_value_words(np.array([g]), w + 1)[0, w])]
                           for g in (0, 1, 12345, 2**40 + 7) for w in (0, 1, 127)],
    }


def synth_case(name, P, B, n, value_len, part_mode, var_len=False, seed=O.SYNTH_SEED) -> dict:
    """A small synthetic build. Fixed-length values unless var_len (len = 1 + w0 % 300)."""
    gids = np.arange(n, dtype=np.uint64)
    kpp = max(1, (n + P - 1) // P)
    parts, bks = O.synth_tags(gids, P, B, part_mode, kpp)
    order, seg_rec = O.layout_a(parts, bks, P, B)
    sg = gids[order]
    if var_len:
        lens = (O.synth_value_words(sg, 1, seed)[:, 0] % np.uint64(300) + np.uint64(1)).astype(np.uint64)
        value_off = np.zeros(n + 1, np.uint64)
        np.cumsum(lens, out=value_off[1:])
        blob = b"".join(bytes(O.synth_values(sg[i:i + 1], int(lens[i]), seed)[0]) for i in range(n))
        values = np.frombuffer(blob, dtype=np.uint8)
    else:
        values = O.synth_values(sg, value_len, seed).reshape(-1)
        value_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(value_len)
    digest, size = O.bucket_digests(values, value_off, seg_rec)
    roots, node_sha, items = [], [], []
    for p in range(P):
        d = [int(x) for x in digest[p * B:(p + 1) * B]]
        levels = O.tree_levels_from_digests(d)
        roots.append(_hex(levels[-1][0]))
        node_sha.append(hashlib.sha256(O.internal_nodes_blob(d)).hexdigest())
        # EpochTreeObject.items walks tree.Leafs: an odd B counts the duplicate leaf twice
        leaf_sizes = [int(x) for x in size[p * B:(p + 1) * B]] + ([int(size[p * B + B - 1])] if B % 2 else [])
        items.append(sum(leaf_sizes))
    # cross-check the array form against the object form (RawPartitionMerkleTree semantics)
    for p in range(min(P, 2)):
        bl = [O.MerkleBucket(b, O.CustomHash()) for b in range(B)]
        for b in range(B):
            s = p * B + b
            for r in range(int(seg_rec[s]), int(seg_rec[s + 1])):
                bl[b].add_item(bytes(values[int(value_off[r]):int(value_off[r + 1])]))
        assert O.new_tree(bl).merkle_root().hex() == roots[p], name
    return {"name": name, "P": P, "B": B, "n": n, "value_len": value_len, "var_len": var_len,
            "part_mode": part_mode, "keys_per_partition": kpp, "seed": seed,
            "seg_rec": [int(x) for x in seg_rec], "digest": [int(x) for x in digest],
            "size": [int(x) for x in size], "items": items, "root": roots, "nodes_sha256": node_sha}


def synth_cases() -> list:
    return [
        synth_case("c1_1p_1000x64_b64", 1, 64, 1000, 64, "block"),
        synth_case("b30_ts8", 2, 30, 600, 8, "mod"),
        synth_case("b1", 3, 1, 90, 16, "mod"),
        synth_case("b2", 2, 2, 50, 24, "mod"),
        synth_case("b3_odd", 2, 3, 70, 33, "mod"),
        synth_case("b7_odd_sparse", 4, 7, 11, 40, "mod"),
        synth_case("b100_hash", 5, 100, 700, 256, "hash"),
        synth_case("b64_unaligned_len13", 4, 64, 900, 13, "mod"),
        synth_case("b64_1k", 8, 64, 512, 1024, "mod"),
        synth_case("b1000", 2, 1000, 3000, 8, "mod"),
        synth_case("var_len", 3, 64, 800, 0, "mod", var_len=True),
        synth_case("empty_partitions", 6, 16, 5, 64, "hash"),
        synth_case("b5000_lds_spill", 1, 5000, 2000, 8, "mod"),
    ]


def diff_cases() -> list:
    rng = np.random.default_rng(7)
    cases = []

    def add(name, d1, d2):
        d1 = [int(x) for x in d1]
        d2 = [int(x) for x in d2]
        try:
            out = O.diff_from_digests(d1, d2)
            exp = {"ids": out}
        except O.MerkleError as e:
            exp = {"error": str(e)}
        cases.append({"name": name, "b1": len(d1), "b2": len(d2), "d1": d1, "d2": d2, **exp})

    for B in (1, 2, 3, 6, 7, 8, 30, 64, 100, 1000):
        base = rng.integers(0, O.HASH_MOD, B)
        add(f"b{B}_equal", base, base)
        one = base.copy(); one[B // 2] = (one[B // 2] + 1) % O.HASH_MOD
        add(f"b{B}_mid", base, one)
        last = base.copy(); last[-1] = (last[-1] + 5) % O.HASH_MOD
        add(f"b{B}_last", base, last)
        alld = (base + 1) % O.HASH_MOD
        add(f"b{B}_all", base, alld)
        rnd = base.copy(); m = rng.random(B) < 0.2; rnd[m] = (rnd[m] + 3) % O.HASH_MOD
        add(f"b{B}_rand", base, rnd)
    # shape mismatches (reference: error or pruned)
    a8 = rng.integers(0, O.HASH_MOD, 8)
    add("b6_vs_b8", a8[:6], a8)
    six = a8[:6].copy(); eight = np.concatenate([six[:4], six[4:6], rng.integers(0, 9, 2)])
    add("b6_vs_b8_prefix_equal", six, eight)
    add("b2_vs_b3", a8[:2], a8[:3])
    add("b3_vs_b4_same_leaves", a8[:3], np.concatenate([a8[:3], a8[2:3]]))
    add("b30_vs_b64", rng.integers(0, 9, 30), rng.integers(0, 9, 64))
    return cases


def main():
    out = {
        "testmerkletreeraw_n100.json": testmerkletreeraw(100),
        "testmerkletreeraw_n10.json": testmerkletreeraw(10),
        "kat_index.json": kat_index(),
        "kat_hash.json": kat_hash(),
        "synth_cases.json": synth_cases(),
        "diff_cases.json": diff_cases(),
    }
    for name, obj in out.items():
        (HERE / name).write_text(json.dumps(obj, indent=None, separators=(",", ":")) + "\n")
        print(f"wrote {name} ({(HERE / name).stat().st_size} bytes)")


if __name__ == "__main__":
    main()
