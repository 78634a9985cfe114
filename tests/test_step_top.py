"""GPU parity of the fused build step's wide trees (plan_step_trees Q = 0: at least 512 partitions
of more than 128 buckets, two waves per tree beside the streaming digest), the production shape's
tree form: every digest, size, item count, internal node and root of every partition must equal the
C oracle's NewTree (cbergoon/merkletree v0.2.0 as restated in oracle/), across runs of pipelined
builds alternating two arenas, partition counts that are not multiples of any grouping, odd bucket
counts and a build without the nodes output. (Written for a grouped pass over the trees' top levels,
measured and rejected in round 4: profiles/r04/r04y_group_top_rejected.txt)"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _arena(P, B, seed, per_bucket=2):
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 2 * per_bucket + 1, P * B).astype(np.uint64)  # some buckets empty
    seg = np.zeros(P * B + 1, np.uint64)
    np.cumsum(counts, out=seg[1:])
    n = int(seg[-1])
    values = rng.integers(1, 1 << 40, n, dtype=np.uint64).view(np.uint8).copy()  # 8-byte timestamps
    return values, seg, n


@pytest.mark.parametrize("P,B", [(512, 1000), (515, 1000), (1027, 1000), (600, 999), (520, 130)])
def test_fused_step_wide_trees_match_oracle(engine, coracle, P, B):
    import torch
    import mydatastore_amd as mde
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    arenas = [_arena(P, B, 11 * P + B + k) for k in range(2)]
    keep, recs = [], []
    for values, seg, n in arenas:
        tv = torch.from_numpy(values).to(dev)
        ts = torch.from_numpy(seg.view(np.int64)).to(dev)
        keep += [tv, ts]
        recs.append(mde.Records(tv.data_ptr(), values.size, 8, mde.LAYOUT_SORTED, 0, n, P, B, ts.data_ptr()))
    NI = O.n_internal_nodes(B)

    def outs(with_nodes):
        o = {"digest": torch.full((P * B,), -1, dtype=torch.int64, device=dev),
             "size": torch.full((P * B,), -1, dtype=torch.int32, device=dev),
             "items": torch.full((P,), -1, dtype=torch.int32, device=dev),
             "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev),
             "nodes": torch.zeros(P * NI * 32, dtype=torch.uint8, device=dev) if with_nodes else None}
        to = mde.TreeOut(*(o[k].data_ptr() if o[k] is not None else 0
                           for k in ("digest", "size", "items", "root", "nodes")))
        return o, to

    # a run of five builds alternating the two arenas: build i's trees run inside build i+1's
    # launch; build 3 without the nodes output
    run = [(k % 2, k != 3) for k in range(5)]
    results = []
    for a, with_nodes in run:
        o, to = outs(with_nodes)
        engine.build_pipelined_async(recs[a], to)
        results.append((a, o))
    engine.build_pipeline_drain_async()
    torch.cuda.synchronize()
    exp = [coracle.build(values, seg, P, B, 8, threads=8) for values, seg, _ in arenas]
    for i, (a, o) in enumerate(results):
        got = {k: (v.cpu().numpy() if v is not None else None) for k, v in o.items()}
        e = exp[a]
        assert np.array_equal(got["digest"].view(np.uint64), e["digest"]), (i, "digest")
        assert np.array_equal(got["size"], e["size"]), (i, "size")
        assert np.array_equal(got["items"], e["items"]), (i, "items")
        assert np.array_equal(got["root"], e["root"]), (i, "root")
        if got["nodes"] is not None:
            assert np.array_equal(got["nodes"], e["nodes"]), (i, "nodes")
