"""GPU parity of the software-pipelined build (mde_build_pipelined_async / _drain_async): one
launch per build that digests build i and builds the trees of build i-1. Every build of a run must
equal the golden fixture (layout A and B, fused and non-fused shapes, empty inputs), whatever the
builds before it were, and the standalone entry points may be interleaved."""
import hashlib

import numpy as np
import pytest

from oracle import oracle as O
from tests.datasets import MODES, synth_arrays

pytestmark = pytest.mark.gpu


def _device_case(case, coracle, layout, dev):
    """Device arrays + Records + outputs for a golden synth case in layout "a" or "b"."""
    import torch
    import mydatastore_amd as mde
    P, B = case["P"], case["B"]
    keep = []

    def up(a):
        t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        keep.append(t)
        return t.data_ptr() if t.numel() else 0

    if layout == "a":
        values, voff, stride, seg = synth_arrays(case, coracle)
        rec = mde.Records(up(values), values.size, stride, mde.LAYOUT_SORTED,
                          up(voff.view(np.int64)) if voff is not None else 0, case["n"], P, B,
                          up(seg.view(np.int64)))
    else:
        n, V = case["n"], case["value_len"]
        gids = np.arange(n, dtype=np.uint64)
        part, bk = coracle.synth_tags(gids, P, B, MODES[case["part_mode"]], case["keys_per_partition"])
        order = np.argsort(part, kind="stable")
        part_rec = np.zeros(P + 1, np.uint64)
        np.cumsum(np.bincount(part, minlength=P), out=part_rec[1:])
        values = coracle.synth_values(gids[order], V, case["seed"])
        tags = bk[order].astype(np.uint16)
        rec = mde.Records(up(values), values.size, V, mde.LAYOUT_TAGGED, 0, n, P, B, 0,
                          up(tags.view(np.int16)), up(part_rec.view(np.int64)))
    o = {"digest": torch.full((P * B,), -1, dtype=torch.int64, device=dev),
         "size": torch.full((P * B,), -1, dtype=torch.int32, device=dev),
         "items": torch.full((P,), -1, dtype=torch.int32, device=dev),
         "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev),
         "nodes": torch.zeros(P * O.n_internal_nodes(B) * 32, dtype=torch.uint8, device=dev)}
    to = mde.TreeOut(*(o[k].data_ptr() for k in ("digest", "size", "items", "root", "nodes")))
    return rec, o, to, keep


def _check(case, o, tag):
    P, B = case["P"], case["B"]
    out = {k: v.cpu().numpy() for k, v in o.items()}
    assert out["digest"].view(np.uint64).tolist() == case["digest"], tag
    assert out["size"].tolist() == case["size"], tag
    assert out["items"].tolist() == case["items"], tag
    assert [out["root"][32 * p:32 * p + 32].tobytes().hex() for p in range(P)] == case["root"], tag
    ni = O.n_internal_nodes(B) * 32
    assert [hashlib.sha256(out["nodes"][p * ni:(p + 1) * ni].tobytes()).hexdigest()
            for p in range(P)] == case["nodes_sha256"], tag


def test_pipelined_run_matches_golden(engine, golden, coracle):
    """All golden cases back to back through the pipeline (each build's trees run inside the next
    build's launch), twice, in layout A and -- where it applies -- layout B, with a standalone
    mde_build_async interleaved mid-run."""
    import torch
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    cases = golden("synth_cases.json")
    run = []
    for rep in range(2):
        for c in cases:
            run.append((c, "a"))
            if not c["var_len"]:
                run.append((c, "b"))
    built = []
    for i, (c, lay) in enumerate(run):
        rec, o, to, keep = _device_case(c, coracle, lay, dev)
        engine.build_pipelined_async(rec, to)
        built.append((c, lay, o, keep))
        if i == len(run) // 2:  # the standalone path shares nothing with the pipeline's scratch
            r2, o2, t2, k2 = _device_case(cases[0], coracle, "a", dev)
            engine.build_async(r2, t2)
            built.append((cases[0], "standalone", o2, k2))
    engine.build_pipeline_drain_async()
    engine.synchronize()
    for c, lay, o, _ in built:
        _check(c, o, (c["name"], lay))


def test_pipelined_drain_is_idempotent_and_single_build(engine, golden, coracle):
    import torch
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    engine.build_pipeline_drain_async()  # nothing pending: no-op
    case = golden("synth_cases.json")[0]
    rec, o, to, keep = _device_case(case, coracle, "a", dev)
    engine.build_pipelined_async(rec, to)
    engine.build_pipeline_drain_async()
    engine.build_pipeline_drain_async()
    engine.synchronize()
    _check(case, o, "single")


def test_pipelined_full_size_equals_standalone(engine):
    """C4 shard of an 8-GPU run (128 partitions x 1 KiB values, 1.28 GB): six pipelined builds
    into alternating output sets equal the standalone build, bit for bit."""
    import torch
    from mydatastore_amd.workload import make_workload
    w = make_workload(engine, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                      n_keys=10_000_000, rank=0, world=8)
    ref = w.build()
    sets = [w._outs() for _ in range(2)]
    for i in range(6):
        if i >= 2:  # output set reused: the build that wrote it is complete in stream order
            for v in sets[i % 2][0].values():
                v.zero_()
        engine.build_pipelined_async(w.rec, sets[i % 2][1])
    engine.build_pipeline_drain_async()
    engine.synchronize()
    for o, _ in sets:
        for k in ("digest", "size", "items", "root", "nodes"):
            assert torch.equal(o[k], ref[k]), k
