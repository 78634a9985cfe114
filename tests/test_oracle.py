"""CPU: the oracle against the reference's own pinned vectors and relations, the golden fixtures,
and the C restatement against the Python restatement."""
import hashlib
import importlib.util

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import GOLDEN, ROOT


def _mtr_manager(n, B=30):
    m = O.Manager(1, B)
    ts = 0
    for i in range(n):
        ts += 1
        m.set_value(f"key{i}", f"val{i}", 1, ts)
    for i in range(n):
        ts += 1
        m.set_value(f"keyz{i}", f"valz{i}", 2, ts)
    return m


@pytest.mark.parametrize("n", [100, 10])
def test_testmerkletreeraw_relations(n):
    """Every assertion of main/merkle_tree_test.go:86-184, on the oracle."""
    m = _mtr_manager(n)
    t1, t2, t3 = (m.raw_partition_merkle_tree(0, lo, 3) for lo in (0, 1, 2))
    for t in (t1, t2, t3):
        assert len(t.leafs) == 30                                    # :86-88
        assert [lf.c.bucket_id for lf in t.leafs] == list(range(30))  # :94-118
    assert t1.merkle_root() == t2.merkle_root()                      # :90
    assert t1.merkle_root() != t3.merkle_root()                      # :91
    assert t2.merkle_root() != t3.merkle_root()                      # :92
    objs = [O.merkle_tree_to_partition_epoch_object(t, 0, lo, 3) for t, lo in ((t1, 0), (t2, 1), (t3, 2))]
    st = [O.epoch_tree_object_to_merkle_tree(o) for o in objs]
    for a, b in zip((t1, t2, t3), st):
        assert a.merkle_root() == b.merkle_root()                    # :150-152
    d1 = O.different_merkle_tree_buckets(t1, t2)
    d2 = O.different_merkle_tree_buckets(t2, t1)
    d3 = O.different_merkle_tree_buckets(t1, t3)
    d4 = O.different_merkle_tree_buckets(t1, st[0])
    d5 = O.different_merkle_tree_buckets(t1, st[2])
    assert d1 == d2 and len(d1) == 0 and d1 == d4                    # :179-181
    assert len(d3) != 0 and len(d5) != 0                             # :183-184


def test_survey_appendix_b():
    """Independently derived values recorded in SURVEY.md Appendix B."""
    m = _mtr_manager(100)
    t1, t3 = m.raw_partition_merkle_tree(0, 0, 3), m.raw_partition_merkle_tree(0, 2, 3)
    assert t1.merkle_root().hex() == "2cb892f8455313dccedb990e7d071816c13c8bb728137c887d2d7c0a3438c7a7"
    assert t3.merkle_root().hex() == "03f02578452d8b229a02a12399d47e105ddbe15ed3e89cb2a2e5ad30e1eacae1"
    assert O.different_merkle_tree_buckets(t1, t3) == list(range(19)) + list(range(20, 30)) + [28, 29]
    assert [lf.c.hasher.hash() for lf in t1.leafs[:6]] == [707, 539, 952, 435, 1041, 703]
    assert [lf.c.size for lf in t1.leafs[:6]] == [6, 7, 8, 6, 7, 8]
    m = _mtr_manager(10)
    assert m.raw_partition_merkle_tree(0, 0, 3).merkle_root().hex() == \
        "5d5f2fb4daa3b70c53ecd56bee99ce02676fbd6b0826706e1fa0c9d7a0186b44"
    assert O.different_merkle_tree_buckets(m.raw_partition_merkle_tree(0, 0, 3),
                                           m.raw_partition_merkle_tree(0, 2, 3)) == [3, 6, 9, 11, 12, 22, 23, 27]


def test_index_kats(golden):
    """main/indexs_test.go:9-41 and storage/index_test.go:9-40 (pinned by the reference)."""
    k = golden("kat_index.json")
    for p, b, e, key, want in k["epoch_index"]:
        assert O.build_epoch_index(p, b, e, key) == want
    for p, e, want in k["epoch_tree_index"]:
        assert O.build_epoch_tree_object_index(p, e) == want
    for name, cols, want in k["generic"]:
        vals = [O._ordered(c[0], c[1]) if isinstance(c, list) else c for c in cols]
        assert O.build_index(name, vals) == want
    for s, p, b, e, key in k["parse"]:
        assert O.parse_epoch_index(s) == (p, b, e, key)
    # ranges never bleed across buckets: '_' (0x5f) sorts after every digit
    assert O.build_epoch_index(0, 10, 1, "x") < O.build_epoch_index(0, 1, 1, "")


def test_hash_kats(golden, coracle):
    k = golden("kat_hash.json")
    assert hashlib.sha256(b"abc").hexdigest().startswith("ba7816bf")
    for m, want in k["sha256"]:
        assert hashlib.sha256(bytes.fromhex(m)).hexdigest() == want
        assert coracle.sha256(bytes.fromhex(m)).hex() == want
    for m, want in k["xxh64_published"] + k["xxh64"]:
        assert "%016x" % O.xxh64(bytes.fromhex(m)) == want
        assert "%016x" % coracle.xxh64(bytes.fromhex(m)) == want
    for key, b64, b1000, p15, p1024 in k["key_tags"]:
        kb = bytes.fromhex(key)
        assert (O.get_key_bucket(kb, 64), O.get_key_bucket(kb, 1000)) == (b64, b1000)
        assert (O.find_partition_id(kb, 15), O.find_partition_id(kb, 1024)) == (p15, p1024)
    for g, w, want in k["splitmix_words"]:
        v = coracle.synth_values(np.array([g], np.uint64), 8 * (w + 1), O.SYNTH_SEED)
        assert "%016x" % int(v[8 * w:8 * w + 8].view("<u8")[0]) == want


def test_customhash_semantics():
    """CustomHash.Add/Remove/Merge (main/merkle_tree.go:25-52): per-record mod == total mod."""
    rng = np.random.default_rng(1)
    recs = [bytes(rng.integers(0, 256, rng.integers(0, 5000), dtype=np.uint8)) for _ in range(300)]
    h = O.CustomHash()
    for r in recs:
        h.add(r)
    assert h.hash() == sum(sum(r) for r in recs) % O.HASH_MOD
    h2 = O.CustomHash(h.hash())
    h2.remove(recs[0])
    assert h2.hash() == (h.hash() - sum(recs[0])) % O.HASH_MOD
    h3 = O.CustomHash(10)
    h3.merge(O.CustomHash(O.HASH_MOD - 3))
    assert h3.hash() == 7


def test_epoch_object_odd_b():
    """Odd B: Leafs include the duplicate, so the wire object carries B+1 buckets (quirk A.2)."""
    t = O.new_tree([O.MerkleBucket(i, O.CustomHash(i * 11), size=i) for i in range(7)])
    obj = O.merkle_tree_to_partition_epoch_object(t, 3, 1, 2)
    assert len(obj.buckets) == 8 and obj.buckets[7] == obj.buckets[6]
    assert obj.items == sum(range(7)) + 6
    rt = O.epoch_tree_object_to_merkle_tree(obj)
    assert rt.merkle_root() == t.merkle_root() and len(rt.leafs) == 8
    with pytest.raises(O.MerkleError):
        O.decode_bytes_to_int64(b"\0" * 7)
    with pytest.raises(O.MerkleError):
        O.new_tree([])


def test_golden_fixtures_regenerate():
    """The committed fixtures are exactly what the committed generator produces."""
    spec = importlib.util.spec_from_file_location("gen_golden", GOLDEN / "gen_golden.py")
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    import json
    assert json.loads((GOLDEN / "testmerkletreeraw_n100.json").read_text()) == \
        json.loads(json.dumps(g.testmerkletreeraw(100)))
    assert json.loads((GOLDEN / "kat_hash.json").read_text()) == json.loads(json.dumps(g.kat_hash()))
    assert json.loads((GOLDEN / "diff_cases.json").read_text()) == json.loads(json.dumps(g.diff_cases()))
    assert json.loads((GOLDEN / "synth_cases.json").read_text()) == json.loads(json.dumps(g.synth_cases()))


def test_c_oracle_build_matches_fixtures(golden, coracle):
    from tests.datasets import synth_arrays
    for case in golden("synth_cases.json"):
        values, voff, stride, seg = synth_arrays(case, coracle)
        for threads in (1, 3):
            out = coracle.build(values, seg, case["P"], case["B"], stride, voff, threads=threads)
            assert out["digest"].tolist() == case["digest"], case["name"]
            assert out["size"].tolist() == case["size"], case["name"]
            assert out["items"].tolist() == case["items"], case["name"]
            roots = [out["root"][32 * p:32 * p + 32].tobytes().hex() for p in range(case["P"])]
            assert roots == case["root"], case["name"]
            ni = O.n_internal_nodes(case["B"]) * 32
            shas = [hashlib.sha256(out["nodes"][p * ni:(p + 1) * ni].tobytes()).hexdigest()
                    for p in range(case["P"])]
            assert shas == case["nodes_sha256"], case["name"]


def test_c_oracle_diff_matches_fixtures(golden, coracle):
    for c in golden("diff_cases.json"):
        got = coracle.diff(c["d1"], c["d2"])
        if "error" in c:
            assert got == -1, c["name"]
        else:
            assert got == c["ids"], c["name"]


def test_testmerkletreeraw_fixture(golden, coracle):
    """Array-form restatement (what the engine computes) == object-form oracle on the reference
    scenario."""
    from tests.datasets import mtr_arena
    for name in ("testmerkletreeraw_n100.json", "testmerkletreeraw_n10.json"):
        fix = golden(name)
        for key, tr in fix["trees"].items():
            lo, hi = map(int, key.split("_"))
            vals, seg = mtr_arena(fix, lo, hi)
            out = coracle.build(vals, seg, 1, fix["n_buckets"], 8)
            assert out["digest"].tolist() == tr["digests"]
            assert out["size"].tolist() == tr["sizes"]
            assert out["root"].tobytes().hex() == tr["root"]
            assert out["nodes"].tobytes().hex() == tr["nodes"]


def test_c_oracle_sha_paths_agree_with_hashlib():
    """oracle/mde_oracle.c hashes on the x86 SHA extensions when the CPU has them (as Go's
    crypto/sha256 does on amd64) and on the portable FIPS 180-4 code otherwise; both equal hashlib
    on every message length around the padding boundaries, and the trees built on them agree."""
    import subprocess
    import sys
    code = r'''
import ctypes, hashlib, json, random, sys
sys.path.insert(0, sys.argv[1])
from tests.oracle_c import COracle
co = COracle()
r = random.Random(7)
for n in list(range(0, 200)) + [4096, 100003]:
    m = bytes(r.getrandbits(8) for _ in range(n))
    assert co.sha256(m) == hashlib.sha256(m).digest(), n
import numpy as np
d = np.array([r.randrange(999999) for _ in range(1000)], np.uint64)
print(json.dumps({"ni": int(co.L.oracle_sha_ni()), "root": co.tree(d, 1000)[0].hex()}))
'''
    import json
    import os
    from tests.conftest import ROOT
    outs = []
    for env in ({}, {"MDE_ORACLE_SHA": "portable"}):
        r = subprocess.run([sys.executable, "-c", code, str(ROOT)], capture_output=True, text=True,
                           env={**os.environ, **env}, timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append(json.loads(r.stdout))
    assert outs[1]["ni"] == 0
    assert outs[0]["root"] == outs[1]["root"]
