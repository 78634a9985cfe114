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


def _variant_ids(engine):
    """The digest-kernel variant ids mde_set_tuning accepts (digest.hip kVariants: 11..16)."""
    import mydatastore_amd as mde
    ids = []
    for v in range(64):
        try:
            engine.set_tuning(v, -1)
            ids.append(v)
        except mde.MdeError:
            pass
    engine.set_tuning(-1, -1)
    return ids


def test_every_digest_variant_matches_golden(engine, golden, coracle):
    """Every digest-kernel variant (one range, pieces, register window, record-space rec8; the
    rec8 ids fall back to the window kernel for other record shapes) through both the standalone
    and the fused path gives the golden outputs."""
    import torch
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ids = _variant_ids(engine)
    assert ids == [11, 12, 13, 14, 15, 16]
    cases = golden("synth_cases.json")
    try:
        for v in ids:
            engine.set_tuning(v, -1)
            built = []
            for c in cases:
                rec, o, to, keep = _device_case(c, coracle, "a", dev)
                engine.build_async(rec, to)
                built.append((c, o, keep))
                rec2, o2, to2, keep2 = _device_case(c, coracle, "a", dev)
                engine.build_pipelined_async(rec2, to2)
                built.append((c, o2, keep2))
            engine.build_pipeline_drain_async()
            engine.synchronize()
            for c, o, _ in built:
                _check(c, o, (c["name"], v))
    finally:
        engine.set_tuning(-1, -1)


def test_every_digest_variant_full_size(engine):
    """C4 at N=1 and the N=8 shard: every variant's roots equal the default build's."""
    import torch
    from mydatastore_amd.workload import make_workload
    ids = _variant_ids(engine)
    for world in (8, 1):
        w = make_workload(engine, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                          n_keys=10_000_000, rank=0, world=world)
        ref = w.build()
        try:
            for v in ids:
                engine.set_tuning(v, -1)
                for _ in range(2):
                    o = w.build()
                    for k in ("digest", "root"):
                        assert torch.equal(o[k], ref[k]), (world, v, k)
        finally:
            engine.set_tuning(-1, -1)
        del w


def test_skewed_arena_every_variant_matches_torch_sums(engine):
    """A 300 MB arena with skew: 13-byte records (never 16-byte aligned), the arena start 5 bytes
    past an allocation, 37 partitions x 100 buckets with empty buckets and partitions and a few
    buckets of tens of MB. Digests of every variant equal per-bucket byte sums computed by torch
    (cumsum over per-record sums) mod 999999."""
    import torch
    import mydatastore_amd as mde
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    g = torch.Generator(device="cpu").manual_seed(7)
    P, B, V = 37, 100, 13
    counts = torch.randint(0, 12_000, (P * B,), generator=g)
    counts[torch.randint(0, P * B, (900,), generator=g)] = 0          # empty buckets
    counts[5 * B:6 * B] = 0                                            # an empty partition
    counts[torch.tensor([17, 1234, 3001])] = torch.tensor([4_000_000, 2_500_000, 3_000_000])
    seg = torch.zeros(P * B + 1, dtype=torch.int64)
    seg[1:] = torch.cumsum(counts, 0)
    n = int(seg[-1])
    buf = torch.randint(0, 256, (n * V + 32,), dtype=torch.uint8, device=dev)
    vals = buf[5:5 + n * V]
    rs = vals.view(n, V).to(torch.int64).sum(1)
    cs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    cs[1:] = torch.cumsum(rs, 0)
    dseg = seg.to(dev)
    want = ((cs[dseg[1:]] - cs[dseg[:-1]]) % 999999).cpu()
    rec = mde.Records(vals.data_ptr(), n * V, V, mde.LAYOUT_SORTED, 0, n, P, B, dseg.data_ptr())
    ids = _variant_ids(engine)
    roots = {}
    try:
        for v in ids:
            engine.set_tuning(v, -1)
            for rep in range(2):
                o = {"digest": torch.zeros(P * B, dtype=torch.int64, device=dev),
                     "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
                     "items": torch.zeros(P, dtype=torch.int32, device=dev),
                     "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev)}
                to = mde.TreeOut(o["digest"].data_ptr(), o["size"].data_ptr(), o["items"].data_ptr(),
                                 o["root"].data_ptr(), 0)
                if rep == 0:
                    engine.build_async(rec, to)
                else:
                    engine.build_pipelined_async(rec, to)
                    engine.build_pipeline_drain_async()
                engine.synchronize()
                assert torch.equal(o["digest"].cpu(), want), (v, rep)
                assert torch.equal(o["size"].cpu().to(torch.int64), counts), (v, rep)
                roots.setdefault("r", o["root"].cpu())
                assert torch.equal(o["root"].cpu(), roots["r"]), (v, rep)
    finally:
        engine.set_tuning(-1, -1)


PIECES_VARIANT = 12  # digest.hip kVariants: U = 4, nontemporal, prefetched, interleaved pieces
WINDOW_VARIANTS = (13, 14)  # the same with the bucket bounds in a register window (14: + pieces)


def _skewed_arena(dev, variable, seed=11, P=37, B=100, max_count=8_000, big=(3_000_000, 1_500_000, 2_000_000),
                  stride=13, start=5):
    """Ragged layout-A arena of ~100-300 MB for the digest work split: empty buckets and an empty
    partition, a few buckets of tens of MB, the arena start `start` bytes past an allocation. Fixed
    `stride`-byte records (13: never 16-byte aligned) or variable lengths 0..40 (value_off). Returns
    the Records, the per-bucket record counts and the expected digests (torch byte sums mod
    999999)."""
    import torch
    import mydatastore_amd as mde
    g = torch.Generator(device="cpu").manual_seed(seed)
    counts = torch.randint(0, max_count, (P * B,), generator=g)
    counts[torch.randint(0, P * B, (P * B // 4,), generator=g)] = 0
    counts[5 * B:6 * B] = 0
    counts[torch.tensor([17, 1234, 3001])] = torch.tensor(list(big))
    seg = torch.zeros(P * B + 1, dtype=torch.int64)
    seg[1:] = torch.cumsum(counts, 0)
    n = int(seg[-1])
    keep = []
    if variable:
        lens = torch.randint(0, 41, (n,), generator=g)
        voff = torch.zeros(n + 1, dtype=torch.int64)
        voff[1:] = torch.cumsum(lens, 0)
        nbytes = int(voff[-1])
        stride = 0
    else:
        nbytes = n * stride
    buf = torch.randint(0, 256, (nbytes + 32,), dtype=torch.uint8, device=dev)
    vals = buf[start:start + nbytes]
    cb = torch.zeros(nbytes + 1, dtype=torch.int64, device=dev)
    cb[1:] = torch.cumsum(vals.to(torch.int64), 0)
    if variable:
        dvoff = voff.to(dev)
        bpos = dvoff[seg.to(dev)]
        keep.append(dvoff)
    else:
        bpos = seg.to(dev) * stride
    want = ((cb[bpos[1:]] - cb[bpos[:-1]]) % 999999).cpu()
    dseg = seg.to(dev)
    keep += [buf, dseg]
    rec = mde.Records(vals.data_ptr(), nbytes, 0 if variable else stride, mde.LAYOUT_SORTED,
                      keep[0].data_ptr() if variable else 0, n, P, B, dseg.data_ptr())
    return rec, counts, want, keep, (P, B)


@pytest.mark.parametrize("variant", [PIECES_VARIANT, WINDOW_VARIANTS[1]])
@pytest.mark.parametrize("variable", [False, True])
def test_digest_pieces_ragged_arena_matches_torch_sums(engine, variable, variant):
    """Interleaved digest pieces (mde_set_digest_piece_bytes) from 1 KiB (a piece switch every
    few steps, pieces ending inside records and buckets) to 1 MiB, and one range per wave: the
    digests equal torch byte sums and the sizes the record counts, standalone and fused."""
    import torch
    import mydatastore_amd as mde
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rec, counts, want, keep, (P, B) = _skewed_arena(dev, variable)
    roots = {}
    engine.set_tuning(variant, -1)
    try:
        for pb in (0, 1024, 3072, 16384, 65536, 1 << 20):
            engine.set_digest_piece_bytes(pb)
            for rep in range(2):
                o = {"digest": torch.zeros(P * B, dtype=torch.int64, device=dev),
                     "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
                     "items": torch.zeros(P, dtype=torch.int32, device=dev),
                     "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev)}
                to = mde.TreeOut(o["digest"].data_ptr(), o["size"].data_ptr(), o["items"].data_ptr(),
                                 o["root"].data_ptr(), 0)
                if rep == 0:
                    engine.build_async(rec, to)
                else:
                    engine.build_pipelined_async(rec, to)
                    engine.build_pipeline_drain_async()
                engine.synchronize()
                assert torch.equal(o["digest"].cpu(), want), (pb, rep)
                assert torch.equal(o["size"].cpu().to(torch.int64), counts), (pb, rep)
                roots.setdefault("r", o["root"].cpu())
                assert torch.equal(o["root"].cpu(), roots["r"]), (pb, rep)
    finally:
        engine.set_digest_piece_bytes(-1)
        engine.set_tuning(-1, -1)


def test_digest_pieces_full_size(engine):
    """C4 at N=1 and the N=8 shard: every piece size gives the roots of one range per wave."""
    import torch
    from mydatastore_amd.workload import make_workload
    for world in (8, 1):
        w = make_workload(engine, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                          n_keys=10_000_000, rank=0, world=world)
        try:
            engine.set_digest_piece_bytes(0)
            ref = w.build()  # default variant, one range per wave
            for v, pb in [(-1, -1)] + [(PIECES_VARIANT, x) for x in (0, 65536, 262144, 1 << 20, 4 << 20)]:
                engine.set_tuning(v, -1)  # (-1, -1): the defaults, automatic pieces
                engine.set_digest_piece_bytes(pb)
                o = w.build()
                for k in ("digest", "size", "root"):
                    assert torch.equal(o[k], ref[k]), (world, pb, k)
        finally:
            engine.set_digest_piece_bytes(-1)
            engine.set_tuning(-1, -1)
        del w


@pytest.mark.parametrize("value_len,n_keys,world,n_buckets", [
    (1024, 10_000_000, 1, 64), (1024, 10_000_000, 8, 64), (100, 4_000_000, 1, 64),
    (8, 20_000_000, 1, 1000), (8, 20_000_000, 8, 64), (16, 10_000_000, 1, 64),
    (1024, 2_000_000, 1, 1000), (2048, 1_000_000, 1, 128), (1024, 10_000_000, 1, 1000),
    (4096, 500_000, 1, 300), (1024, 4_000_000, 8, 1000), (1024, 3_000_000, 1, 4000)])
def test_tagged_equals_layout_a_full_size(engine, value_len, n_keys, world, n_buckets):
    """Layout B (arrival order + bucket tags, binned on device), standalone and fused: digests,
    sizes, items and roots equal the layout-A build of the same records, at C4 (N=1 and the N=8
    shard). 100-byte values put record boundaries inside the 16-byte vectors (the general
    binning path); 8- and 16-byte values take the small-record path (the production timestamp
    size), at B = 64 and the reference's default B = 1000. 1, 2 and 4 KiB values at B = 128 to
    4,000 take the row-reduced fast step (fewer than 64 lane slots per bucket: 32 down to 1; C4 at
    B = 1,000 whole, and its N = 8 shard)."""
    import torch
    from mydatastore_amd.workload import make_workload
    kw = dict(n_partitions=1024, n_buckets=n_buckets, value_len=value_len, part_mode="mod", n_keys=n_keys,
              rank=0, world=world)
    wa = make_workload(engine, layout="a", **kw)
    ref = wa.build()
    del wa
    wb = make_workload(engine, layout="b", **kw)
    for fused in (False, True):
        if fused:
            o, to = wb._outs()
            engine.build_pipelined_async(wb.rec, to)
            engine.build_pipeline_drain_async()
            engine.synchronize()
        else:
            o = wb.build()
        for k in ("digest", "size", "items", "root"):
            assert torch.equal(o[k], ref[k]), (fused, k)


@pytest.mark.parametrize("layout,n_buckets,world", [
    ("a", 1000, 1), ("b", 1000, 1), ("a", 1000, 8), ("b", 1000, 8), ("a", 64, 1), ("b", 64, 1)])
def test_fused_step_trees_many_builds(engine, layout, n_buckets, world):
    """Runs of pipelined builds, where every build but the last gets its trees from the NEXT
    build's launch (the fused step's tree workgroups): 1,024 partitions (two-wave trees at
    B = 1,000) and the 128-partition N = 8 shard (packed tree waves), 8-byte values, both layouts.
    Every build of the run equals the standalone build, nodes included."""
    import torch
    from mydatastore_amd.workload import make_workload
    w = make_workload(engine, n_partitions=1024, n_buckets=n_buckets, value_len=8, part_mode="mod",
                      n_keys=20_000_000, rank=0, world=world, layout=layout)
    ref = w.build()
    sets = [w._outs() for _ in range(3)]
    for o, to in sets:
        engine.build_pipelined_async(w.rec, to)
    engine.build_pipeline_drain_async()
    engine.synchronize()
    for i, (o, _) in enumerate(sets):
        for k in ("digest", "size", "items", "root", "nodes"):
            assert torch.equal(o[k], ref[k]), (i, k)


@pytest.mark.parametrize("P,n_buckets", [(131, 129), (131, 257), (3, 999), (131, 1000), (512, 1023), (1, 1024)])
def test_whole_workgroup_step_trees_match_oracle(engine, coracle, P, n_buckets):
    """Few wide trees beside a short stream (plan_step_trees' whole-workgroup form, r06: the
    production shape's N = 8 shard): the fused step's trees over all 256 threads of a workgroup,
    the upper half as schedule helpers -- odd and even B, the level of <= 128 nodes that starts the
    split levels (129, 257), the fused step's LDS limit (1,024), 1 to 512 partitions. A run of
    pipelined builds equals the C oracle, nodes included."""
    import numpy as np
    import torch
    from mydatastore_amd.workload import make_workload
    V = 8
    w = make_workload(engine, n_partitions=P, n_buckets=n_buckets, value_len=V, part_mode="mod",
                      n_keys=min(300 * P, 1_500_000), rank=0, world=1, layout="a")
    exp = coracle.build(w.values.cpu().numpy(), w.seg_rec.cpu().numpy().view(np.uint64), P, n_buckets,
                        stride=V, threads=8)
    sets = [w._outs() for _ in range(3)]
    for o, to in sets:
        engine.build_pipelined_async(w.rec, to)
    engine.build_pipeline_drain_async()
    engine.synchronize()
    for i, (o, _) in enumerate(sets):
        for k in ("digest", "size", "items", "root", "nodes"):
            got = o[k].cpu().numpy().view(exp[k].dtype).reshape(-1)
            assert np.array_equal(got, exp[k].reshape(-1)), (i, k)


@pytest.mark.parametrize("n_buckets", [129, 257, 999, 1000, 1024])
def test_pair_trees_odd_shapes_match_oracle(engine, coracle, n_buckets):
    """Wide trees of >= 512 partitions: the standalone tree kernel's pair shape (two partitions
    per workgroup) and the fused step's two-wave trees. An odd partition count (the last pair
    workgroup holds one live tree), odd B (duplicate leaf, self-paired nodes), B whose level 2
    already fits one wave (129) or needs one wide level (257), and the fused step's LDS limit
    (1,024). The standalone build and a pipelined run equal the C oracle, nodes included."""
    import numpy as np
    import torch
    from mydatastore_amd.workload import make_workload
    P, V = 515, 8
    w = make_workload(engine, n_partitions=P, n_buckets=n_buckets, value_len=V, part_mode="mod",
                      n_keys=1_500_000, rank=0, world=1, layout="a")
    exp = coracle.build(w.values.cpu().numpy(), w.seg_rec.cpu().numpy().view(np.uint64), P, n_buckets,
                        stride=V, threads=8)
    outs = [w.build()]
    sets = [w._outs() for _ in range(2)]
    for o, to in sets:
        engine.build_pipelined_async(w.rec, to)
    engine.build_pipeline_drain_async()
    engine.synchronize()
    outs += [o for o, _ in sets]
    for i, o in enumerate(outs):
        for k in ("digest", "size", "items", "root", "nodes"):
            got = o[k].cpu().numpy().view(exp[k].dtype).reshape(-1)
            assert np.array_equal(got, exp[k].reshape(-1)), (i, k)


@pytest.mark.parametrize("variable", [False, True])
def test_many_small_buckets_every_static_variant(engine, variable):
    """The reference's default PartitionBuckets = 1000 (config/default-config.yaml:8) with a few
    records per bucket: a wave crosses a bucket boundary every few hundred bytes, so every window
    reload and every crossing inside a 16-byte vector is exercised. 64 partitions x 1000 buckets,
    0-19 records of 13 bytes (or 0-40-byte variable records) per bucket, a quarter empty, an empty
    partition and three buckets of a few MB: every static variant (one range, pieces, register
    window, both; pieces from 1 KiB) equals torch byte sums, standalone and fused."""
    import torch
    import mydatastore_amd as mde
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rec, counts, want, keep, (P, B) = _skewed_arena(dev, variable, seed=5, P=64, B=1000, max_count=20,
                                                    big=(300_000, 200_000, 250_000))
    try:
        for v in (11, PIECES_VARIANT) + WINDOW_VARIANTS:
            engine.set_tuning(v, -1)
            for pb in ((-1, 1024, 8192) if v in (PIECES_VARIANT, WINDOW_VARIANTS[1]) else (-1,)):
                engine.set_digest_piece_bytes(pb)
                for fused in (False, True):
                    o = {"digest": torch.zeros(P * B, dtype=torch.int64, device=dev),
                         "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
                         "items": torch.zeros(P, dtype=torch.int32, device=dev),
                         "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev)}
                    to = mde.TreeOut(o["digest"].data_ptr(), o["size"].data_ptr(), o["items"].data_ptr(),
                                     o["root"].data_ptr(), 0)
                    if fused:
                        engine.build_pipelined_async(rec, to)
                        engine.build_pipeline_drain_async()
                    else:
                        engine.build_async(rec, to)
                    engine.synchronize()
                    assert torch.equal(o["digest"].cpu(), want), (v, pb, fused)
                    assert torch.equal(o["size"].cpu().to(torch.int64), counts), (v, pb, fused)
    finally:
        engine.set_digest_piece_bytes(-1)
        engine.set_tuning(-1, -1)


@pytest.mark.parametrize("value_len,n_keys,n_buckets,world", [
    (1024, 10_000_000, 1000, 1), (1024, 10_000_000, 1000, 8), (8, 20_000_000, 1000, 1),
    (8, 20_000_000, 64, 1), (64, 4_000_000, 1000, 1), (13, 6_000_000, 1000, 1)])
def test_default_variant_choice_b1000_full_size(engine, value_len, n_keys, n_buckets, world):
    """The reference's default PartitionBuckets = 1000 (C4: 10 KiB buckets) and production-sized
    values (8-byte timestamps: ~160 B buckets, several bucket starts per step, the prefix-scan
    path; 13-byte records: starts inside vectors): the automatic choice (the register-window
    kernel, pieces for large shares) gives exactly what the round-1 kernel (variant 11, one range
    per wave) gives, standalone and fused."""
    import torch
    from mydatastore_amd.workload import make_workload
    w = make_workload(engine, n_partitions=1024, n_buckets=n_buckets, value_len=value_len, part_mode="mod",
                      n_keys=n_keys, rank=0, world=world)
    try:
        engine.set_tuning(11, -1)
        engine.set_digest_piece_bytes(0)
        ref = w.build()
        engine.set_tuning(-1, -1)
        engine.set_digest_piece_bytes(-1)
        for fused in (False, True):
            if fused:
                o, to = w._outs()
                engine.build_pipelined_async(w.rec, to)
                engine.build_pipeline_drain_async()
                engine.synchronize()
            else:
                o = w.build()
            for k in ("digest", "size", "items", "root", "nodes"):
                assert torch.equal(o[k], ref[k]), (fused, k)
    finally:
        engine.set_tuning(-1, -1)
        engine.set_digest_piece_bytes(-1)


# digest.hip: fixed 8-byte records, record-space prefix scan (+ pieces)
REC8_VARIANTS = (15, 16)
REC8_PIECES = (16,)


@pytest.mark.parametrize("start", [0, 8])
@pytest.mark.parametrize("P,B,max_count", [(37, 1000, 300), (64, 64, 3000)])
def test_rec8_ragged_arena_matches_torch_sums(engine, coracle, start, P, B, max_count):
    """The 8-byte-record digest (production timestamps, main/manager.go:816): 37 or 64 partitions, a
    quarter of the buckets empty, an empty partition, three buckets of 12-24 MB (past the 16 MiB
    exact-u32 reduction), the arena 16-byte aligned or 8 bytes past it (record slots on 8-byte
    boundaries), both variants and piece sizes from 1 KiB (piece and range ends inside buckets and
    in the middle of 16-byte vectors), standalone and fused: digests equal torch byte sums, sizes
    the record counts, items their per-partition sums, roots the C oracle's SHA-256 trees over
    those digests, and the automatic choice picks it."""
    import torch
    import mydatastore_amd as mde
    dev = torch.device("cuda:0")
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rec, counts, want, keep, (P, B) = _skewed_arena(dev, False, seed=3 + start, P=P, B=B, max_count=max_count,
                                                    big=(3_000_000, 1_500_000, 2_000_000), stride=8, start=start)
    want_np = want.numpy().astype(np.uint64)
    want_root = torch.from_numpy(np.concatenate(
        [np.frombuffer(coracle.tree(want_np[p * B:(p + 1) * B], B)[0], np.uint8) for p in range(P)]).copy())
    want_items = counts.view(P, B).sum(1).to(torch.int32)
    try:
        for v, pbs in [(-1, (-1,))] + [(v, (1024, 8192, 1 << 20) if v in REC8_PIECES else (-1,))
                                       for v in REC8_VARIANTS]:
            engine.set_tuning(v, -1)
            for pb in pbs:
                engine.set_digest_piece_bytes(pb)
                for fused in (False, True):
                    o = {"digest": torch.zeros(P * B, dtype=torch.int64, device=dev),
                         "size": torch.zeros(P * B, dtype=torch.int32, device=dev),
                         "items": torch.zeros(P, dtype=torch.int32, device=dev),
                         "root": torch.zeros(P * 32, dtype=torch.uint8, device=dev)}
                    to = mde.TreeOut(o["digest"].data_ptr(), o["size"].data_ptr(), o["items"].data_ptr(),
                                     o["root"].data_ptr(), 0)
                    if fused:
                        engine.build_pipelined_async(rec, to)
                        engine.build_pipeline_drain_async()
                    else:
                        engine.build_async(rec, to)
                    engine.synchronize()
                    assert torch.equal(o["digest"].cpu(), want), (v, pb, fused)
                    assert torch.equal(o["size"].cpu().to(torch.int64), counts), (v, pb, fused)
                    assert torch.equal(o["items"].cpu(), want_items), (v, pb, fused)
                    assert torch.equal(o["root"].cpu(), want_root), (v, pb, fused)
    finally:
        engine.set_digest_piece_bytes(-1)
        engine.set_tuning(-1, -1)
