"""Seeded randomized parity: many random build shapes through the C ABI against the C oracle.

Each case draws P, B, the record counts per bucket (zero-heavy, skewed), the value layout (fixed
stride 1..2048 B incl. odd and power-of-two strides, or variable 0..600 B), arena misalignment,
and the entry point (host mde_build, device mde_build_async, pipelined, layout B for fixed
strides). Every output is compared bit for bit: digests, sizes, items, roots, all internal nodes.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# MDE_FUZZ_SEED / MDE_FUZZ_CASES override the seed and case count for longer one-off runs
N_CASES = int(os.environ.get("MDE_FUZZ_CASES", "160"))
SEED = int(os.environ.get("MDE_FUZZ_SEED", "20261016"))
MAX_BYTES = 96 << 20  # per case; the C oracle checks it on one host thread


def _case(rng):
    P = int(rng.choice([1, 2, 3, 7, 16, 33]))
    B = int(rng.choice([1, 2, 3, 5, 16, 30, 64, 100, 257, 1000]))
    S = P * B
    dist = rng.integers(0, 3)
    if dist == 0:      # sparse: most buckets empty
        counts = rng.integers(0, 6, S) * (rng.random(S) < 0.2)
    elif dist == 1:    # uniform
        counts = rng.integers(0, 40, S)
    else:              # skewed: a few huge buckets
        counts = rng.integers(0, 4, S)
        hot = rng.choice(S, size=max(1, S // 20), replace=False)
        counts[hot] = rng.integers(200, 3000, hot.size)
    var = bool(rng.random() < 0.3)
    stride = 0 if var else int(rng.choice([1, 3, 8, 13, 16, 64, 100, 256, 1024, 2048]))
    est = int(counts.sum()) * (300 if var else stride)
    if est > MAX_BYTES:
        counts = counts * MAX_BYTES // est
    return P, B, counts.astype(np.uint64), var, stride


def _arrays(rng, counts, var, stride):
    n = int(counts.sum())
    seg = np.zeros(counts.size + 1, np.uint64)
    np.cumsum(counts, out=seg[1:])
    if var:
        lens = rng.integers(0, 601, n).astype(np.uint64)
        voff = np.zeros(n + 1, np.uint64)
        np.cumsum(lens, out=voff[1:])
        vals = rng.integers(0, 256, int(voff[-1]), dtype=np.uint8)
        return vals, voff, seg
    return rng.integers(0, 256, n * stride, dtype=np.uint8), None, seg


def _dev_outs(torch, mde, P, B, dev):
    o = {"digest": torch.full((P * B,), -1, dtype=torch.int64, device=dev),
         "size": torch.full((P * B,), -1, dtype=torch.int32, device=dev),
         "items": torch.full((P,), -1, dtype=torch.int32, device=dev),
         "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev),
         "nodes": torch.zeros(P * mde.tree_internal_nodes(B) * 32, dtype=torch.uint8, device=dev)}
    return o, mde.TreeOut(*(o[k].data_ptr() for k in ("digest", "size", "items", "root", "nodes")))


CHECKED = []


def _cmp(got, exp, tag):
    CHECKED.append(tag)
    for k in ("digest", "size", "items", "root", "nodes"):
        g = np.asarray(got[k])
        e = np.asarray(exp[k])
        assert np.array_equal(g.view(e.dtype) if g.dtype != e.dtype and g.itemsize == e.itemsize else g, e), (tag, k)


def test_random_builds_match_oracle(engine, coracle):
    import torch
    import mydatastore_amd as mde
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rng = np.random.default_rng(SEED)
    pending = []
    for i in range(N_CASES):
        P, B, counts, var, stride = _case(rng)
        vals, voff, seg = _arrays(rng, counts, var, stride)
        exp = coracle.build(vals, seg, P, B, stride, voff)
        tag = (i, P, B, var, stride, int(counts.sum()))
        path = i % 4
        if path == 0:  # host API
            _cmp(engine.build(vals, seg, P, B, stride, voff), exp, tag)
            continue
        shift = int(rng.integers(0, 16))
        buf = torch.zeros(vals.size + 32, dtype=torch.uint8, device=dev)
        if vals.size:
            buf[shift:shift + vals.size] = torch.from_numpy(vals).to(dev)
        dv = buf[shift:shift + vals.size]
        n = int(counts.sum())
        if path == 3 and not var and stride:  # layout B: records of each partition shuffled
            part = np.repeat(np.arange(P), [int(counts[p * B:(p + 1) * B].sum()) for p in range(P)])
            bk = np.concatenate([np.repeat(np.arange(B), counts[p * B:(p + 1) * B].astype(np.int64))
                                 for p in range(P)]) if n else np.zeros(0, np.int64)
            perm = np.concatenate([rng.permutation(np.flatnonzero(part == p)) for p in range(P)]) if n else \
                np.zeros(0, np.int64)
            rec_vals = vals.reshape(n, stride)[perm].reshape(-1) if n else vals
            tags = bk[perm].astype(np.uint16)
            part_rec = np.zeros(P + 1, np.uint64)
            np.cumsum(np.bincount(part, minlength=P), out=part_rec[1:])
            buf2 = torch.zeros(rec_vals.size + 32, dtype=torch.uint8, device=dev)
            if rec_vals.size:
                buf2[shift:shift + rec_vals.size] = torch.from_numpy(np.ascontiguousarray(rec_vals)).to(dev)
            dv2 = buf2[shift:shift + rec_vals.size]
            dt = torch.from_numpy(tags.view(np.int16)).to(dev)
            dp = torch.from_numpy(part_rec.view(np.int64)).to(dev)
            rec = mde.Records(dv2.data_ptr() if n else 0, rec_vals.size, stride, mde.LAYOUT_TAGGED, 0, n, P, B,
                              0, dt.data_ptr() if n else 0, dp.data_ptr())
            keep = (buf2, dt, dp)
        else:
            dseg = torch.from_numpy(seg.view(np.int64)).to(dev)
            dvo = torch.from_numpy(voff.view(np.int64)).to(dev) if var else None
            rec = mde.Records(dv.data_ptr() if vals.size else 0, vals.size, stride, mde.LAYOUT_SORTED,
                              dvo.data_ptr() if var else 0, n, P, B, dseg.data_ptr())
            keep = (dseg, dvo)
        o, to = _dev_outs(torch, mde, P, B, dev)
        if path == 2:  # pipelined: outputs complete after the next pipelined call or the drain
            engine.build_pipelined_async(rec, to)
            pending.append((o, exp, tag, keep, buf))
            if len(pending) == 3:
                engine.build_pipeline_drain_async()
                engine.synchronize()
                for po, pe, pt, _, _ in pending:
                    _cmp({k: v.cpu().numpy() for k, v in po.items()}, pe, pt)
                pending.clear()
            continue
        engine.build_async(rec, to)
        engine.synchronize()
        _cmp({k: v.cpu().numpy() for k, v in o.items()}, exp, tag)
    engine.build_pipeline_drain_async()
    engine.synchronize()
    for po, pe, pt, _, _ in pending:
        _cmp({k: v.cpu().numpy() for k, v in po.items()}, pe, pt)
    assert len(CHECKED) == N_CASES
    print(f"{N_CASES} cases, {sum(t[-1] for t in CHECKED)} records")
