"""Output staging of the synchronous host calls (csrc/mde_api.cpp HostIo): write-once outputs are
stored by the kernels straight into pinned staging memory (the default); MDE_DIRECT_OUT=0 copies
them back with a D2H copy instead. Both must give the same bytes -- and the oracle's -- for builds
(B <= 4,096: every output direct; wider trees re-read their node levels, so their outputs stay in
device memory) and for the decision step (valid and the peer statuses stay in device memory: the
fold and the encode read them again)."""
import numpy as np
import pytest

from tests.test_verify import STATUS, _oracle_verify, _peer_objects


@pytest.fixture()
def copy_engine(monkeypatch):
    import mydatastore_amd as mde
    monkeypatch.setenv("MDE_DIRECT_OUT", "0")  # read when the context is created
    eng = mde.Engine(0)
    monkeypatch.delenv("MDE_DIRECT_OUT")
    yield eng
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("B,n,stride", [(64, 3000, 8), (1000, 20000, 8), (1000, 5000, 0), (5000, 30000, 13)])
def test_build_outputs_direct_equal_copied_and_oracle(engine, copy_engine, coracle, B, n, stride):
    rng = np.random.default_rng(B + n)
    P = 3
    lens = np.full(n, stride) if stride else rng.integers(0, 40, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    vals = rng.integers(0, 256, int(off[-1]) or 1, dtype=np.uint8)
    seg = np.concatenate([[0], np.sort(rng.integers(0, n + 1, P * B - 1)), [n]]).astype(np.uint64)
    kw = dict(value_stride=stride) if stride else dict(value_off=off)
    a = engine.build(vals, seg, P, B, **kw)
    b = copy_engine.build(vals, seg, P, B, **kw)
    want = coracle.build(vals, seg, P, B, stride, None if stride else off)
    for k in ("digest", "size", "items", "root", "nodes"):
        assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(a[k], want[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1], ids=["fused", "chain"])
@pytest.mark.parametrize("B", [64, 1000])
def test_verify_outputs_direct_equal_copied_and_oracle(engine, copy_engine, B, mode):
    rng = np.random.default_rng(7 * B + mode)
    P, E, replica = 8, 5, 2
    digests = rng.integers(0, 999999, size=P * B, dtype=np.uint64)
    sizes = rng.integers(0, 5000, size=P * B).astype(np.int32)
    parts = (np.arange(P) * 5 + 1).astype(np.int32)
    peers = [_peer_objects(rng, B, digests[p * B:(p + 1) * B], sizes[p * B:(p + 1) * B], int(parts[p]), E)
             for p in range(P)]
    res = []
    for eng in (engine, copy_engine):
        eng.set_verify_mode(mode)
        try:
            res.append(eng.verify_epochs(B, digests, sizes, None, peers, replica, E, partition=parts))
        finally:
            eng.set_verify_mode(0)
    want = _oracle_verify(B, digests, sizes, peers, replica, E, parts)
    for p in range(P):
        for got in res:
            assert got["valid"][p] == want[p]["valid"]
            assert got["valid_count"][p] == want[p]["valid_count"]
            assert got["diff"][p] == want[p]["diff"]
            assert got["peer_status"][p] == [STATUS.get(x, x) for x in want[p]["status"]]
            assert got["objects"][p] == want[p]["object"]
