"""Seeded random shapes through the fused pipelined build (mde_build_pipelined_async: one
build_step_kernel launch per build, carrying the previous build's trees) and the standalone build,
device-resident, against the C oracle: partition counts 1-300, B from 1 to 1,000, fixed-length
values of 1-1,024 bytes (the 8-byte record scan among them) or variable lengths 0-70 bytes, arenas
starting at a 16-byte boundary or 8 bytes past it, empty buckets and partitions. Each case runs two
different builds back to back in one pipeline, so launch 2 builds the first build's trees while it
streams the second's records, and checks both builds' digests, sizes, items, roots and nodes."""
import numpy as np
import pytest


def _cases(k, seed=777):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        P = int(rng.choice([1, 2, 7, 64, 300]))
        B = int(rng.choice([1, 2, 3, 5, 64, 65, 129, 333, 1000]))
        V = int(rng.choice([0, 1, 3, 8, 8, 16, 24, 64, 100, 1024]))  # 0: variable lengths
        per = int(rng.choice([0, 1, 5, 20]))
        n = max(0, min(400_000, int(P * B * per * rng.uniform(0.5, 1.5))))
        if V == 1024:
            n = min(n, 60_000)
        out.append((P, B, V, n, int(rng.integers(0, 2)) * 8, int(rng.integers(0, 1 << 30))))
    return out


def _records(rng, P, B, V, n):
    S = P * B
    cuts = np.sort(rng.integers(0, n + 1, S - 1)) if S > 1 else np.zeros(0, np.int64)
    seg = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    if V:
        return rng.integers(0, 256, n * V, dtype=np.uint8), seg, None
    lens = rng.integers(0, 71, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return rng.integers(0, 256, int(off[-1]), dtype=np.uint8), seg, off


@pytest.mark.gpu
@pytest.mark.parametrize("P,B,V,n,shift,seed", _cases(16))
def test_fused_pipeline_random_shapes_match_oracle(engine, coracle, P, B, V, n, shift, seed):
    import torch
    import mydatastore_amd as mde
    rng = np.random.default_rng(seed)
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ni = mde.tree_internal_nodes(B)
    builds, keep = [], []
    for _ in range(2):
        vals, seg, off = _records(rng, P, B, V, n)
        # the arena `shift` bytes into its allocation (16-byte aligned + 0 or 8)
        buf = torch.zeros(vals.size + shift + 16, dtype=torch.uint8, device=dev)
        buf[shift:shift + vals.size].copy_(torch.from_numpy(vals))
        d_seg = torch.from_numpy(seg.view(np.int64)).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev) if off is not None else None
        base = buf.data_ptr() + shift
        rec = mde.Records(base if vals.size else 0, vals.size, V, mde.LAYOUT_SORTED,
                          d_off.data_ptr() if d_off is not None else 0, n, P, B, d_seg.data_ptr())
        o = {"digest": torch.zeros(P * B, dtype=torch.int64, device=dev),
             "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
             "items": torch.zeros(P, dtype=torch.int32, device=dev),
             "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev),
             "nodes": torch.zeros(P * ni * 32, dtype=torch.uint8, device=dev)}
        to = mde.TreeOut(*(o[k].data_ptr() for k in ("digest", "size", "items", "root", "nodes")))
        exp = coracle.build(vals, seg, P, B, stride=V, value_off=off)
        builds.append((rec, o, to, exp))
        keep.append((buf, d_seg, d_off))
    for rec, o, to, exp in builds:  # two builds in one pipeline
        engine.build_pipelined_async(rec, to)
    engine.build_pipeline_drain_async()
    engine.synchronize()
    for i, (rec, o, to, exp) in enumerate(builds):
        assert np.array_equal(o["digest"].cpu().numpy().view(np.uint64), exp["digest"]), ("digest", i)
        assert np.array_equal(o["size"].cpu().numpy(), exp["size"]), ("size", i)
        assert np.array_equal(o["items"].cpu().numpy(), exp["items"]), ("items", i)
        assert np.array_equal(o["root"].cpu().numpy(), exp["root"]), ("root", i)
        assert np.array_equal(o["nodes"].cpu().numpy(), exp["nodes"]), ("nodes", i)
    # the standalone build of the second records, into fresh outputs
    rec, o, to, exp = builds[1]
    for t in o.values():
        t.zero_()
    engine.build_async(rec, to)
    engine.synchronize()
    assert np.array_equal(o["root"].cpu().numpy(), exp["root"])
    assert np.array_equal(o["nodes"].cpu().numpy(), exp["nodes"])


@pytest.mark.gpu
@pytest.mark.parametrize("P,B,V,n,shift,seed", [c for c in _cases(12, seed=4242) if c[2]])
def test_tagged_pipeline_random_shapes_match_oracle(engine, coracle, P, B, V, n, shift, seed):
    """Layout B (records grouped by partition in arrival order, one u16 bucket tag each, binned on
    the device): the same random shapes (fixed-length values) through two pipelined builds, against
    the C oracle's build of the records sorted by (partition, bucket) -- a bucket's digest, size
    and item count do not depend on its records' order."""
    import torch
    import mydatastore_amd as mde
    rng = np.random.default_rng(seed)
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ni = mde.tree_internal_nodes(B)
    builds, keep = [], []
    for _ in range(2):
        cuts = np.sort(rng.integers(0, n + 1, P - 1)) if P > 1 else np.zeros(0, np.int64)
        part_rec = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
        tags = rng.integers(0, B, n).astype(np.uint16)
        vals = rng.integers(0, 256, n * V, dtype=np.uint8)
        # the oracle's layout A: stable sort by (partition, tag)
        part_of = np.repeat(np.arange(P), np.diff(part_rec).astype(np.int64))
        order = np.lexsort((tags, part_of)) if n else np.zeros(0, np.int64)
        sorted_vals = vals.reshape(n, V)[order].reshape(-1) if n else vals
        counts = np.bincount(part_of * B + tags.astype(np.int64), minlength=P * B) if n else np.zeros(P * B, np.int64)
        seg = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
        exp = coracle.build(sorted_vals, seg, P, B, stride=V)
        buf = torch.zeros(vals.size + shift + 16, dtype=torch.uint8, device=dev)
        buf[shift:shift + vals.size].copy_(torch.from_numpy(vals))
        d_tag = torch.from_numpy(tags.view(np.int16).copy()).to(dev)
        d_pr = torch.from_numpy(part_rec.view(np.int64)).to(dev)
        rec = mde.Records(buf.data_ptr() + shift if vals.size else 0, vals.size, V, mde.LAYOUT_TAGGED, 0, n, P, B, 0,
                          d_tag.data_ptr() if n else 0, d_pr.data_ptr())
        o = {"digest": torch.zeros(P * B, dtype=torch.int64, device=dev),
             "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
             "items": torch.zeros(P, dtype=torch.int32, device=dev),
             "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev),
             "nodes": torch.zeros(P * ni * 32, dtype=torch.uint8, device=dev)}
        to = mde.TreeOut(*(o[k].data_ptr() for k in ("digest", "size", "items", "root", "nodes")))
        builds.append((rec, o, to, exp))
        keep.append((buf, d_tag, d_pr))
    for rec, o, to, exp in builds:
        engine.build_pipelined_async(rec, to)
    engine.build_pipeline_drain_async()
    engine.synchronize()
    for i, (rec, o, to, exp) in enumerate(builds):
        assert np.array_equal(o["digest"].cpu().numpy().view(np.uint64), exp["digest"]), ("digest", i)
        assert np.array_equal(o["size"].cpu().numpy(), exp["size"]), ("size", i)
        assert np.array_equal(o["items"].cpu().numpy(), exp["items"]), ("items", i)
        assert np.array_equal(o["root"].cpu().numpy(), exp["root"]), ("root", i)
        assert np.array_equal(o["nodes"].cpu().numpy(), exp["nodes"]), ("nodes", i)
