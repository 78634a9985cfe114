"""The resident build service (mde_server_build, include/mde.h): one-partition builds -- the
reference's production call shape, one RawPartitionMerkleTree per (partition, epoch) from
VerifyEpoch (main/manager.go:1036, main/merkle_tree.go:86-116) on up to partition_concurrency = 10
workers (config/default-config.yaml:9) -- served by a persistent launch polling request slots in
pinned host memory. Every caller's result equals mde_build's and the C oracle's; the launch ends
at its lifetime and relaunches without losing a request."""
import json
import subprocess
import threading

import numpy as np
from pathlib import Path
import pytest

from tests.conftest import ROOT

BIN = ROOT / "tests" / "cpp" / "build" / "server_test"


def test_server_test_builds_and_fails_loudly_without_gpu():
    import torch
    assert BIN.exists()
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([str(BIN), "2", "1"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "mde_server_create: -3" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("threads,calls,lifetime_ms", [(10, 40, 100), (1, 8, 100), (32, 8, 100), (8, 30, 2)])
def test_server_concurrent_callers_c(threads, calls, lifetime_ms):
    """tests/cpp/server_test.c: `threads` pthreads released together, each making `calls` builds
    (B = 1 / 2 / 30 / 64 / 1000 / 1024 in the service, 4096 and > 256 KiB inputs on its context;
    8-byte, variable-length and uniform variable-length values; records outside the bucket ranges;
    empty partitions; 2-3 partitions per call; full, root-only and digest-only outputs). Every
    output == mde_build == the C oracle. A 2 ms lifetime relaunches the service while calls are in
    flight; the last calls each find the launch ended (idle past the lifetime)."""
    r = subprocess.run([str(BIN), str(threads), str(calls), str(lifetime_ms)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])["server_test"]
    assert d["mismatches"] == 0 and d["calls"] == threads * calls + 6
    assert d["idle_relaunches_ok"]
    assert d["on_context"] < d["requests"]  # most calls ran in the resident workgroups
    if lifetime_ms <= 2:
        assert d["launches"] > 6, d


@pytest.mark.gpu
def test_server_python_threads_match_oracle(coracle):
    """Ten Python threads (ctypes releases the GIL) on one Server: 8-byte timestamp records at the
    reference's default B = 1000 and at B = 64, full and digest-only builds; every result equals
    the C oracle's build."""
    import mydatastore_amd as mde
    sv = mde.Server(0)
    errors = []

    def caller(t):
        rng = np.random.default_rng(300 + t)
        try:
            for k in range(12):
                B = (64, 1000)[(t + k) % 2]
                n = int(rng.integers(200, 4000))
                ts = rng.integers(1, 1 << 40, n, dtype=np.uint64)
                vals = ts.view(np.uint8).copy()  # LE64 timestamps (main/manager.go:816)
                cuts = np.sort(rng.integers(0, n + 1, B - 1))
                seg = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
                tree = k % 3 != 2
                got = sv.build(vals, seg, 1, B, value_stride=8, want_tree=tree)
                exp = coracle.build(vals, seg, 1, B, 8)
                for key in ("digest", "size", "items") + (("root", "nodes") if tree else ()):
                    if not np.array_equal(got[key], exp[key]):
                        errors.append((t, k, key))
        except Exception as e:  # pragma: no cover
            errors.append((t, repr(e)))

    ths = [threading.Thread(target=caller, args=(t,)) for t in range(10)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    st = sv.stats()
    sv.close()
    assert not errors, errors[:5]
    assert st["requests"] == 10 * 12 and st["on_context"] == 0


@pytest.mark.gpu
def test_server_python_decisions_match_oracle(coracle):
    """The VerifyEpoch decision step through the service (Server.verify) from eight Python
    threads at B = 64 and 1000: agreeing, one-bucket-differing, absent and garbage peers; every
    result equals the oracle's VerifyEpoch restatement (oracle.py verify_epoch,
    main/manager.go:1072-1104)."""
    import mydatastore_amd as mde
    from oracle import oracle as O
    from oracle import wire_pb
    sv = mde.Server(0)
    errors = []

    def caller(t):
        rng = np.random.default_rng(700 + t)
        try:
            for k in range(10):
                B = (64, 1000)[(t + k) % 2]
                n = int(rng.integers(200, 3000))
                ts = rng.integers(1, 1 << 40, n, dtype=np.uint64)
                vals = ts.view(np.uint8).copy()
                cuts = np.sort(rng.integers(0, n + 1, B - 1))
                seg = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
                exp = coracle.build(vals, seg, 1, B, 8)
                d = exp["digest"].astype(np.uint64)
                z = exp["size"]
                d2 = d.copy()
                d2[(3 * k + t) % B] = (d2[(3 * k + t) % B] + 1) % 999999
                peers = [wire_pb.marshal(5, 2, 3, d.tolist(), z.tolist()),
                         wire_pb.marshal(5, 2, 3, d2.tolist(), z.tolist(), valid=bool(k % 2)),
                         None, b"\xff\xff"]
                res = sv.verify(B, d, z, peers, replica_count=2, epoch=2, partition=5)
                want = O.verify_epoch(O.tree_from_digests(d.tolist(), z.tolist()), 5, 2, peers, 2)
                if (res["valid"], res["valid_count"], res["diff"], res["object"]) != \
                        (want["valid"], want["valid_count"], want["diff"], want["object"]):
                    errors.append((t, k))
        except Exception as e:  # pragma: no cover
            errors.append((t, repr(e)))

    ths = [threading.Thread(target=caller, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    st = sv.stats()
    sv.close()
    assert not errors, errors[:5]
    assert st["requests"] == 8 * 10 and st["on_context"] == 0


@pytest.mark.gpu
def test_two_live_services_on_one_device_do_not_queue_behind_each_other(coracle):
    """Two services alive on one device at once, each with its own caller thread: each launch runs
    on a kept stream no other live service holds, so neither waits for the other's lifetime
    (default 100 ms) -- every call returns in well under that; every result equals the oracle."""
    import time
    import mydatastore_amd as mde
    svs = [mde.Server(0), mde.Server(0)]
    worst, errors = [0.0, 0.0], []

    def caller(t):
        rng = np.random.default_rng(900 + t)
        try:
            for k in range(40):
                n = int(rng.integers(100, 2000))
                vals = rng.integers(1, 1 << 40, n, dtype=np.uint64).view(np.uint8).copy()
                seg = np.concatenate([[0], np.sort(rng.integers(0, n + 1, 63)), [n]]).astype(np.uint64)
                t0 = time.perf_counter()
                got = svs[t].build(vals, seg, 1, 64, value_stride=8)
                worst[t] = max(worst[t], time.perf_counter() - t0)
                exp = coracle.build(vals, seg, 1, 64, 8)
                if not (np.array_equal(got["root"], exp["root"]) and np.array_equal(got["digest"], exp["digest"])):
                    errors.append((t, k))
        except Exception as e:  # pragma: no cover
            errors.append((t, repr(e)))

    try:
        ths = [threading.Thread(target=caller, args=(t,)) for t in range(2)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    finally:
        for sv in svs:
            sv.close()
    assert not errors, errors[:5]
    assert max(worst) < 0.05, worst


@pytest.mark.gpu
@pytest.mark.parametrize("B", [64, 1000, 1023])
def test_server_levels_plus_host_top_equals_oracle(coracle, B):
    """The split tree (mde_server_build_levels): the device's levels down to the first of at most
    64 nodes, the top levels hashed here with hashlib (node = SHA256(left || right), an odd level's
    last node paired with itself, merkletree v0.2.0's rule); every node and the root equal the
    oracle's tree."""
    import hashlib
    import mydatastore_amd as mde
    rng = np.random.default_rng(B)
    n = 3000
    vals = rng.integers(1, 1 << 40, n, dtype=np.uint64).view(np.uint8).copy()
    seg = np.concatenate([[0], np.sort(rng.integers(0, n + 1, B - 1)), [n]]).astype(np.uint64)
    sv = mde.Server(0)
    try:
        got = sv.build_levels(vals, seg, 1, B, 64, value_stride=8)
    finally:
        sv.close()
    exp = coracle.build(vals, seg, 1, B, 8)
    nodes = got["nodes"].reshape(-1, 32).copy()
    pre = got["prefix_nodes"]
    assert np.array_equal(nodes[:pre], exp["nodes"].reshape(-1, 32)[:pre])
    assert not nodes[pre:].any()
    sizes, m = [], (B + 1) // 2  # level sizes, level 1 .. the root
    while True:
        sizes.append(m)
        if m == 1:
            break
        m = (m + 1) // 2
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
    for k in range(1, len(sizes)):
        if offs[k] < pre:
            continue  # a level the device wrote (the prefix covers whole levels)
        for j in range(sizes[k]):
            left, right = 2 * j, min(2 * j + 1, sizes[k - 1] - 1)
            msg = nodes[offs[k - 1] + left].tobytes() + nodes[offs[k - 1] + right].tobytes()
            nodes[offs[k] + j] = np.frombuffer(hashlib.sha256(msg).digest(), np.uint8)
    assert np.array_equal(nodes.reshape(-1), exp["nodes"]) and np.array_equal(nodes[-1], exp["root"])
    assert np.array_equal(got["digest"], exp["digest"]) and np.array_equal(got["size"], exp["size"])


def test_tree_prefix_nodes_matches_level_walk():
    """CPU: mde_tree_prefix_nodes (what mde_server_build_levels writes per partition) is the node
    count of levels 1 .. the first level of at most top_nodes nodes, merkletree v0.2.0's level
    sizes (level 1 = ceil(B / 2), the odd duplicate leaf included; each next level ceil(n / 2));
    top <= 1 gives every level (mde_tree_internal_nodes)."""
    import ctypes
    lib = ctypes.CDLL(str(ROOT / "mydatastore_amd" / "libmde.so"))
    lib.mde_tree_prefix_nodes.restype = ctypes.c_uint64
    lib.mde_tree_prefix_nodes.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    lib.mde_tree_internal_nodes.restype = ctypes.c_uint64
    lib.mde_tree_internal_nodes.argtypes = [ctypes.c_uint32]
    for B in list(range(1, 300)) + [511, 512, 513, 1000, 1023, 1024, 4096, 65536]:
        for top in (0, 1, 2, 3, 16, 63, 64, 65, 300, 100000):
            t, n = 0, (B + 1) // 2
            stop = max(top, 1)
            while True:
                t += n
                if n <= stop:
                    break
                n = (n + 1) // 2
            assert lib.mde_tree_prefix_nodes(B, top) == t, (B, top)
        assert lib.mde_tree_prefix_nodes(B, 0) == lib.mde_tree_internal_nodes(B)


@pytest.mark.gpu
@pytest.mark.parametrize("B,n", [(2000, 3000), (1000, 40000)])
def test_server_levels_on_the_service_context(coracle, B, n):
    """mde_server_build_levels for a request the resident workgroups do not take -- B beyond the
    launch's 1,024 buckets, or more than 256 KiB of packed inputs -- runs as mde_build on the
    service's context: the prefix of levels the caller reads equals the oracle's nodes (the nodes
    past it are unspecified there: that path writes every level)."""
    import mydatastore_amd as mde
    rng = np.random.default_rng(B + n)
    vals = rng.integers(1, 1 << 40, n, dtype=np.uint64).view(np.uint8).copy()
    seg = np.concatenate([[0], np.sort(rng.integers(0, n + 1, B - 1)), [n]]).astype(np.uint64)
    sv = mde.Server(0)
    try:
        before = sv.stats()["on_context"]
        got = sv.build_levels(vals, seg, 1, B, 64, value_stride=8)
        assert sv.stats()["on_context"] == before + 1
    finally:
        sv.close()
    exp = coracle.build(vals, seg, 1, B, 8)
    pre = got["prefix_nodes"]
    assert np.array_equal(got["nodes"].reshape(-1, 32)[:pre], exp["nodes"].reshape(-1, 32)[:pre])
    assert np.array_equal(got["digest"], exp["digest"]) and np.array_equal(got["size"], exp["size"])
    assert np.array_equal(got["items"], exp["items"])


@pytest.mark.gpu
def test_disable_ends_the_resident_launch():
    """mde_server_disable posts the stop word to the idle slots, so the persistent launch gives its
    CUs back at once instead of polling until its lifetime ends: with a 60 s lifetime, a service
    disabled after serving a call is destroyed in well under a second (a launch left running would
    hold mde_server_destroy for its 10 s bound and keep its buffers)."""
    import subprocess
    import sys
    code = (
        "import time, numpy as np, mydatastore_amd as mde\n"
        "sv = mde.Server(0)\n"
        "vals = np.arange(800, dtype=np.uint8)\n"
        "seg = np.array([0, 40, 100], np.uint64)\n"
        "sv.build(vals, seg, 1, 2, value_stride=8)\n"
        "assert sv.stats()['on_context'] == 0\n"
        "sv.disable('test')\n"
        "time.sleep(0.2)\n"
        "t0 = time.perf_counter()\n"
        "sv.close()\n"
        "print('CLOSE', time.perf_counter() - t0)\n")
    import os
    env = dict(os.environ, MDE_SERVER_LIFETIME_MS="60000")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=100, env=env,
                       cwd=str(Path(__file__).resolve().parents[1]))
    assert r.returncode == 0, r.stderr
    dt = float(r.stdout.split("CLOSE")[1])
    assert dt < 1.0 and "did not end" not in r.stderr, (dt, r.stderr)


@pytest.mark.gpu
def test_disabled_service_serves_every_call_on_its_context(coracle):
    """Once the resident launch is out of service (mde_server_disable here; a failed launch or a
    30 s request timeout take the same path) every later build and decision runs on the service's
    context instead of failing, with the oracle's results, from concurrent callers."""
    from oracle import oracle as O
    from oracle import wire_pb
    import mydatastore_amd as mde
    sv = mde.Server(0)
    try:
        assert sv.usable
        sv.disable("test")
        assert not sv.usable
        errors = []

        def caller(t):
            try:
                rng = np.random.default_rng(100 + t)
                for k in range(4):
                    B = (64, 1000)[k % 2]
                    n = 1000
                    vals = rng.integers(1, 1 << 40, n, dtype=np.uint64).view(np.uint8).copy()
                    seg = np.concatenate([[0], np.sort(rng.integers(0, n + 1, B - 1)), [n]]).astype(np.uint64)
                    got = sv.build(vals, seg, 1, B, value_stride=8)
                    exp = coracle.build(vals, seg, 1, B, 8)
                    for key in ("digest", "size", "items", "root", "nodes"):
                        if not np.array_equal(got[key], exp[key]):
                            errors.append((t, k, key))
                    d = [int(x) for x in exp["digest"]]
                    z = [int(x) for x in exp["size"]]
                    peer = list(d)
                    peer[3] = (peer[3] + 1) % 999999
                    tree = O.tree_from_digests(peer, z)
                    obj = O.merkle_tree_to_partition_epoch_object(tree, 5, 2, 3)
                    blob = wire_pb.marshal(5, 2, 3, [O.decode_bytes_to_int64(h) for h in obj.buckets],
                                           obj.buckets_size, valid=False, items=obj.items)
                    v = sv.verify(B, exp["digest"], exp["size"], [blob, None], 2, 2, partition=5)
                    w = O.verify_epoch(O.tree_from_digests(d, z), 5, 2, [blob, None], 2)
                    if (v["valid"] != w["valid"] or v["valid_count"] != w["valid_count"] or v["diff"] != w["diff"]
                            or v["object"] != w["object"]):
                        errors.append((t, k, "verify"))
            except Exception as e:  # noqa: BLE001
                errors.append((t, repr(e)))

        th = [threading.Thread(target=caller, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:5]
        st = sv.stats()
        assert st["on_context"] == st["requests"] == 32
    finally:
        sv.close()


def _random_server_cases(k, seed=5150):
    """Seeded random one-call shapes: 1-4 partitions, B from 1 to 1,500 (some past the service's
    slot limits, which run on its context), fixed 8-byte or variable-length values (0-40 bytes,
    empty buckets and empty values among them)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        P = int(rng.integers(1, 5))
        B = int(rng.choice([1, 2, 3, 7, 64, 65, 333, 1000, 1500]))
        fixed = bool(rng.integers(0, 2))
        n = int(rng.integers(0, 3000))
        out.append((P, B, fixed, n, int(rng.integers(0, 1 << 30))))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("P,B,fixed,n,seed", _random_server_cases(12))
def test_server_random_shapes_match_oracle(coracle, P, B, fixed, n, seed):
    """The resident service over seeded random shapes, full trees and digest-only builds, every
    output equal to the C oracle's build of the same records (whatever served it: a resident slot
    or, for the shapes past its slot limits, the service's context)."""
    import mydatastore_amd as mde
    rng = np.random.default_rng(seed)
    S = P * B
    cuts = np.sort(rng.integers(0, n + 1, S - 1)) if S > 1 else np.zeros(0, np.int64)
    seg = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    if fixed:
        vals = rng.integers(0, 256, n * 8, dtype=np.uint8)
        kw, okw = {"value_stride": 8}, {"stride": 8}
    else:
        lens = rng.integers(0, 41, n)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        vals = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
        kw, okw = {"value_off": off}, {"value_off": off}
    exp = coracle.build(vals, seg, P, B, **okw)
    sv = mde.Server(0)
    try:
        for tree in (True, False):
            got = sv.build(vals, seg, P, B, want_tree=tree, **kw)
            for key in ("digest", "size", "items") + (("root", "nodes") if tree else ()):
                assert np.array_equal(got[key], exp[key]), (key, tree)
    finally:
        sv.close()
