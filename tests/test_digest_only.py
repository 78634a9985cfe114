"""Digest-only builds (mde_tree_out.root == NULL, include/mde.h): RawPartitionMerkleTree's bucket
digests, sizes and items (main/merkle_tree.go:86-113,121-134) without the SHA-256 tree, for a
caller that builds its tree on the host (the Go shim with mdeHostTree). Every path that can take
one -- the one-launch small build, the digest kernels + leaves kernel, layout B, the batcher --
returns exactly the C oracle's outputs, and a full build on the same inputs agrees."""
import threading

import numpy as np
import pytest


def _arena(rng, P, B, n, stride):
    """P partitions of n records each (layout A), random bucket cuts, some buckets empty."""
    seg = np.zeros(P * B + 1, np.uint64)
    for p in range(P):
        cuts = np.sort(rng.integers(0, n + 1, B - 1))
        seg[p * B + 1:(p + 1) * B] = p * n + cuts
        seg[(p + 1) * B] = (p + 1) * n
    if stride:
        values = rng.integers(0, 256, P * n * stride, dtype=np.uint8)
        return values, seg, None
    lens = rng.integers(0, 40, P * n)
    voff = np.zeros(P * n + 1, np.uint64)
    np.cumsum(lens, out=voff[1:])
    values = rng.integers(0, 256, int(voff[-1]) + 1, dtype=np.uint8)
    return values, seg, voff


SHAPES = [  # (P, B, records per partition, stride): small-build and streaming kernels, odd B, wide B
    (1, 1, 50, 8), (1, 30, 1000, 8), (7, 31, 300, 0), (3, 64, 2000, 64), (300, 64, 100, 8),
    (5, 1000, 5000, 8), (2, 5000, 20000, 8), (64, 1000, 40000, 8), (4, 64, 300000, 16),
]


@pytest.mark.gpu
@pytest.mark.parametrize("P,B,n,stride", SHAPES)
def test_digest_only_build_equals_oracle(engine, coracle, P, B, n, stride):
    rng = np.random.default_rng(P * 7919 + B * 31 + n)
    values, seg, voff = _arena(rng, P, B, n, stride)
    got = engine.build(values, seg, P, B, stride, voff, want_tree=False)
    assert got["root"] is None and got["nodes"] is None
    exp = coracle.build(values, seg, P, B, stride, voff, want_nodes=False)
    for k in ("digest", "size", "items"):
        assert np.array_equal(got[k], exp[k]), k
    full = engine.build(values, seg, P, B, stride, voff, want_nodes=False)
    assert np.array_equal(full["root"], exp["root"])
    assert np.array_equal(full["digest"], got["digest"])


@pytest.mark.gpu
@pytest.mark.parametrize("B", [63, 1000])
def test_digest_only_layout_b_equals_oracle(engine, coracle, B):
    """Layout B (records in write order + bucket tags): the tagged digest kernel + leaves kernel."""
    rng = np.random.default_rng(B)
    P, n, stride = 9, 4000, 8
    tags = rng.integers(0, B, P * n).astype(np.uint16)
    values = rng.integers(0, 256, P * n * stride, dtype=np.uint8)
    part_rec = np.arange(P + 1, dtype=np.uint64) * n
    got = engine.build_tagged(values, part_rec, tags, P, B, stride, want_tree=False)
    # the same records in layout A (stable sort by (partition, bucket)) for the oracle
    key = np.repeat(np.arange(P), n) * B + tags
    order = np.argsort(key, kind="stable")
    seg = np.zeros(P * B + 1, np.uint64)
    np.cumsum(np.bincount(key, minlength=P * B), out=seg[1:])
    va = values.reshape(-1, stride)[order].reshape(-1)
    exp = coracle.build(va, seg, P, B, stride, None, want_nodes=False)
    for k in ("digest", "size", "items"):
        assert np.array_equal(got[k], exp[k]), k


@pytest.mark.gpu
def test_digest_only_batched_with_full_builds(coracle):
    """Eight threads on one batcher, alternating digest-only and full one-partition builds (they
    batch apart: a digest-only request never waits for a tree); every result equals the oracle."""
    import mydatastore_amd as mde
    bt = mde.Batcher(0)
    errors = []

    def caller(t):
        rng = np.random.default_rng(500 + t)
        try:
            for k in range(10):
                B = (64, 1000, 30)[(t + k) % 3]
                values, seg, voff = _arena(rng, 1, B, int(rng.integers(1, 3000)), 8)
                tree = (t + k) % 2 == 0
                got = bt.build(values, seg, 1, B, 8, voff, want_nodes=tree, want_tree=tree)
                exp = coracle.build(values, seg, 1, B, 8, voff)
                keys = ("digest", "size", "items") + (("root", "nodes") if tree else ())
                for key in keys:
                    if not np.array_equal(got[key], exp[key]):
                        errors.append((t, k, key))
        except Exception as e:  # pragma: no cover - reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=caller, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    bt.close()
    assert not errors, errors[:5]


@pytest.mark.gpu
def test_nodes_without_root_rejected(engine):
    import mydatastore_amd as mde
    values = np.zeros(64, np.uint8)
    seg = np.array([0, 4, 8], np.uint64)
    rec = mde.Records(values.ctypes.data, 64, 8, 0, 0, 8, 1, 2, seg.ctypes.data)
    nodes = np.zeros(32 * 8, np.uint8)
    out = mde.TreeOut(0, 0, 0, 0, nodes.ctypes.data)
    import ctypes
    rc = engine.lib.mde_build(engine.ctx, ctypes.byref(rec), ctypes.byref(out))
    assert rc == mde.MDE_E_INVAL
