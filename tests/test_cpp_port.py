"""The C++ port of the reference's Merkle tests (tests/cpp/test_merkle_tree.cpp) over the host
mirror + engine; its printed roots and diffs must equal the golden fixtures."""
import subprocess
import sys

import pytest

from tests.conftest import ROOT

BIN = ROOT / "tests" / "cpp" / "build" / "test_merkle_tree"


def test_cpp_port_builds():
    subprocess.run([sys.executable, "-m", "mydatastore_amd._build", "-q"], cwd=ROOT, check=True)
    assert BIN.exists()
    assert (ROOT / "mydatastore_amd" / "libmde_host.so").exists()


@pytest.mark.gpu
def test_cpp_port_matches_golden(golden):
    r = subprocess.run([str(BIN)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = {(ln.split()[0], ln.split()[1]): (ln.split()[2] if len(ln.split()) > 2 else "")
             for ln in r.stdout.splitlines() if ln.startswith(("ROOT", "DIFF", "ITEMS", "WIRE"))}
    for n in (100, 10):
        fix = golden(f"testmerkletreeraw_n{n}.json")
        for key in ("0_3", "1_3", "2_3"):
            assert lines[("ROOT", f"n{n}_{key}")] == fix["trees"][key]["root"]
        assert lines[("DIFF", f"n{n}_t1_t3")] == ",".join(map(str, fix["diffs"]["t1_t3"]))
        assert int(lines[("ITEMS", f"n{n}_0_3")]) == fix["trees"]["0_3"]["items"]
        assert lines[("WIRE", f"n{n}_0_3")] == fix["trees"]["0_3"]["wire"]
    assert "PASS" in r.stdout
    stream = {ln.split()[1]: ln.split()[2:] for ln in r.stdout.splitlines() if ln.startswith("STREAM")}
    for n in (100, 10):  # TestStreamBucketsTask: 2N records in [0,3); the subset equals its buckets
        total, sub, want = map(int, stream[f"n{n}"])
        assert total == 2 * n and sub == want
    # the request-order list b1, 99, b0, b1, 1000 against the oracle's StreamBucketsTask
    # (main/manager.go:445-487): repeats streamed again, 1000 (>= B) streams nothing
    seq = {ln.split()[1]: ln.split()[2:] for ln in r.stdout.splitlines() if ln.startswith("STREAMSEQ")}
    for n in (100, 10):
        from oracle import oracle as O
        m = O.Manager(1, 100)
        for i in range(n):
            m.set_value(f"key{i}", f"val{i}", 1, 0)
        for i in range(n):
            m.set_value(f"keyz{i}", f"valz{i}", 2, 0)
        allrec = m.stream_buckets(0, [], 0, 3)
        b0 = O.get_key_bucket(allrec[0][0].encode(), 100)
        b1 = O.get_key_bucket(allrec[-1][0].encode(), 100)
        assert seq[f"n{n}"][:2] == [str(b0), str(b1)]
        want = [f"{k}:{e}:{t}" for k, e, t in m.stream_buckets(0, [b1, 99, b0, b1, 1000], 0, 3)]
        assert seq[f"n{n}"][2:] == want
    got = {ln.split()[1]: ln.split()[2:] for ln in r.stdout.splitlines() if ln.startswith("VERIFY")}
    for name, res in _verify_expected().items():
        diff = ",".join(map(str, res["diff"]))
        assert got[name] == [str(int(res["valid"])), str(res["valid_count"])] + ([diff] if diff else []), name


def _verify_expected():
    """The TestVerifyEpoch scenario of tests/cpp/test_merkle_tree.cpp on the oracle."""
    from oracle import oracle as O
    from oracle import wire_pb
    a, b, c = (O.Manager(1, 16) for _ in range(3))
    for i in range(40):
        for m in (a, b) + ((c,) if i < 35 else ()):
            m.set_value(f"key{i}", f"val{i}", 1, i + 1)
    for i in range(3):
        c.set_value(f"other{i}", "x", 1, 100 + i)
    trees = {k: m.raw_partition_merkle_tree(0, 1, 2) for k, m in (("a", a), ("b", b), ("c", c))}

    def wire(t):
        o = O.merkle_tree_to_partition_epoch_object(t, 0, 1, 2)
        return wire_pb.marshal(0, 1, 2, [O.decode_bytes_to_int64(h) for h in o.buckets], o.buckets_size)

    oa, ob, oc = (wire(trees[k]) for k in "abc")
    res = {"a_r3": O.verify_epoch(trees["a"], 0, 1, [oa, ob, oc], 3)}
    res["a_r2"] = O.verify_epoch(trees["a"], 0, 1, [oa, ob, oc], 2)
    res["c_vd"] = O.verify_epoch(trees["c"], 0, 1, [oc, res["a_r2"]["object"], b"\xff"], 3)
    res["b_r2"] = O.verify_epoch(trees["b"], 0, 1, [oa, oc], 2)
    return res


C_BENCH = ROOT / "tests" / "cpp" / "build" / "cabi_bench"


def test_cabi_bench_fails_loudly_without_gpu():
    """The plain-C driver of include/mde.h builds, and without a gfx950 device it stops at
    mde_create with MDE_E_DEVICE (there is no CPU fallback behind the ABI)."""
    import torch
    subprocess.run([sys.executable, "-m", "mydatastore_amd._build", "-q"], cwd=ROOT, check=True)
    assert C_BENCH.exists()
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([str(C_BENCH), "1000", "4", "64", "8", "2", "1"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 1 and "mde_create" in r.stderr and "-3" in r.stderr


@pytest.mark.gpu
def test_cabi_bench_parity():
    """A reduced C4-shaped workload (1M keys, 256 partitions x 256 B values) driven from C without
    PyTorch: roots == tree(digests), sampled bucket digests == host byte sums of the records
    copied back, pipelined timed-run roots == standalone roots."""
    import json
    r = subprocess.run([str(C_BENCH), "1000000", "256", "256", "64", "4", "1"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(ln) for ln in r.stdout.strip().splitlines()]
    d = lines[0]
    assert all(d["parity"].values()), d
    assert d["device"].startswith("gfx950")
    assert [x["records"] for x in lines[1:4]] == [1000, 10000, 100000]
    assert lines[4]["verify_ok"], lines[4]  # one agreeing peer, one differing in bucket 0
