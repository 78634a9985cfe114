"""GPU parity of the split-schedule trees (tree_body_duo): the latency form that the one-partition
calls, small batches and the fused step's wide trees use. Every tree shape boundary of the form --
level-1 widths around the group sizes (8 .. 64 lanes, one wave, a 256-thread workgroup), the first
split level (<= 128 / <= 64 nodes), odd levels -- against the C oracle, bit-exact, roots and every
internal node; and launches past kDuoMaxBlocks, which take the plain tree_body form."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SHAPES = (1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 130, 200, 255, 256,
          257, 258, 511, 512, 513, 767, 768, 999, 1000, 1001, 2047, 2048, 4095, 4096)


def _check_trees(engine, coracle, d, B, T):
    root, nodes = engine.tree_from_digests(d, B)
    ni = O.n_internal_nodes(B) * 32
    for t in range(T):
        r, n = coracle.tree(d[t * B:(t + 1) * B], B)
        assert root[32 * t:32 * t + 32].tobytes() == r, (B, T, t)
        assert nodes[t * ni:(t + 1) * ni].tobytes() == n, (B, T, t)


@pytest.mark.parametrize("T", [1, 2, 5])
def test_duo_tree_from_digests_every_shape(engine, coracle, T):
    rng = np.random.default_rng(100 + T)
    for B in SHAPES:
        d = rng.integers(0, 2**63, T * B, dtype=np.int64).astype(np.uint64)
        _check_trees(engine, coracle, d, B, T)


def test_duo_and_plain_launch_shapes(engine, coracle):
    """Narrow trees past kDuoMaxBlocks workgroups (plain tree_body) and just under it (split
    schedule), plus wide trees under the pair-kernel threshold (split schedule, 511 trees)."""
    rng = np.random.default_rng(7)
    for B, T in ((64, 2 * 256), (64, 2 * 256 + 1), (8, 8 * 256 + 3), (200, 511)):
        d = rng.integers(0, 2**63, T * B, dtype=np.int64).astype(np.uint64)
        _check_trees(engine, coracle, d, B, T)


@pytest.mark.parametrize("P", [1, 3, 9])
def test_duo_small_build_every_shape(engine, coracle, P):
    """One-launch small builds (small_build_kernel, split-schedule trees): 8-byte timestamps like
    the production call, random bucket boundaries including empty buckets."""
    rng = np.random.default_rng(200 + P)
    for B in SHAPES:
        if B > 1024 and P > 1:
            continue
        n = int(rng.integers(0, 3 * B + 2)) * P
        vals = rng.integers(0, 1 << 62, n, dtype=np.uint64).view(np.uint8).copy()
        seg = np.concatenate([[0], np.sort(rng.integers(0, n + 1, P * B - 1)), [n]]).astype(np.uint64)
        out = engine.build(vals, seg, P, B, 8)
        exp = coracle.build(vals, seg, P, B, 8, None)
        for k in ("digest", "size", "items", "root", "nodes"):
            assert np.array_equal(out[k], exp[k]), (B, P, k)
