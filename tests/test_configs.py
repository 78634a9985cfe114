"""GPU parity of the BASELINE.json configurations at full size (configs[1..4]; configs[0], the
reference's CPU case, is the golden fixture c1 in test_gpu_parity.py).

Each full-size build is checked three independent ways:
  * every bucket digest and size against torch byte sums of the device arena (per-record sums,
    prefix sums, differences at the bucket bounds, mod 999999) -- a computation that shares no
    code with the engine's kernels;
  * every root against the C oracle's SHA-256 tree over those digests;
  * a sample of partitions against the C oracle's whole build (oracle/mde_oracle.c) on records
    REGENERATED ON THE HOST by the oracle's own generator (tests/sample.py), i.e. also checking
    the device-side workload generator -- the same sample bench.py's cpu_baseline leg uses.
Both the standalone build (mde_build_async) and the fused pipelined build the bench times
(mde_build_pipelined_async) are checked.

C5 (anti-entropy diff): C4 data as replica A, replica B with one bucket per partition perturbed;
the device DFS diff of every partition is exactly that bucket and the range extract returns
exactly replica B's records of it (indices, offsets and bytes), as bench.py --config c5 times it.
Reference: main/merkle_tree.go:86-216, main/manager.go:445-487 (StreamBucketsTask).
"""
import numpy as np
import pytest

from tests.sample import host_sample, perturb_first_record

pytestmark = pytest.mark.gpu

# BASELINE.json configs (bench.py CONFIGS): n_keys, P, value_len, B, partition mode
C2 = (25_600_000, 256, 256, 64, "block")
C3 = (64_000_000, 64, 1024, 64, "block")
C4 = (10_000_000, 1024, 1024, 64, "mod")
# The reference's own default shapes (not BASELINE configs): partition_buckets = 1000
# (config/default-config.yaml:10). PROD is the production value shape -- every epoch-index record's
# value is the 8-byte LE write timestamp (main/manager.go:816) -- 100M of them over 1,024
# partitions, the bench's production_shape line; C4K is C4 at B = 1000.
PROD = (100_000_000, 1024, 8, 1000, "mod")
C4K = (10_000_000, 1024, 1024, 1000, "mod")


def _torch_digests(w):
    """Exact digests and sizes of every bucket of a layout-A workload, from torch byte sums."""
    import torch
    V, n = w.value_len, w.n_records
    dev = w.values.device
    cs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    step = 1 << 18  # records per chunk: bounds any widened temporary to 2 GiB at 1 KiB values
    for i in range(0, n, step):
        j = min(n, i + step)
        cs[i + 1:j + 1] = w.values[i * V:j * V].view(j - i, V).sum(1, dtype=torch.int64)
    cs = torch.cumsum(cs, 0)
    seg = w.seg_rec
    dig = ((cs[seg[1:]] - cs[seg[:-1]]) % 999999).cpu().numpy().astype(np.uint64)
    size = (seg[1:] - seg[:-1]).to(torch.int32).cpu().numpy()
    return dig, size


def _check_full(o, w, exp_dig, exp_size, coracle, tag):
    P, B = w.n_partitions, w.n_buckets
    got = {k: v.cpu().numpy() for k, v in o.items()}
    assert np.array_equal(got["digest"].view(np.uint64), exp_dig), tag
    assert np.array_equal(got["size"], exp_size), tag
    assert np.array_equal(got["items"], exp_size.reshape(P, B).sum(1, dtype=np.int64).astype(np.int32)), tag
    roots = np.concatenate([np.frombuffer(coracle.tree(exp_dig[p * B:(p + 1) * B], B)[0], np.uint8)
                            for p in range(P)])
    assert np.array_equal(got["root"], roots), tag


def _check_sample(o, w, ref, n, tag):
    B = w.n_buckets
    got = {k: v.cpu().numpy() for k, v in o.items()}
    assert np.array_equal(got["digest"][:n * B].view(np.uint64), ref["digest"]), tag
    assert np.array_equal(got["size"][:n * B], ref["size"]), tag
    assert np.array_equal(got["items"][:n], ref["items"]), tag
    assert np.array_equal(got["root"][:n * 32], ref["root"]), tag
    assert np.array_equal(got["nodes"][:n * ref["nodes"].size // n], ref["nodes"]), tag


def _builds(engine, w):
    """The standalone build and a fused pipelined run of two builds (the bench's timed shape)."""
    outs = [("standalone", w.build())]
    sets = [w._outs() for _ in range(2)]
    for _, to in sets:
        engine.build_pipelined_async(w.rec, to)
    engine.build_pipeline_drain_async()
    engine.synchronize()
    return outs + [(f"fused{i}", o) for i, (o, _) in enumerate(sets)]


@pytest.mark.parametrize("cfg,sample", [(C2, [0, 1, 255]), (C3, [0, 63]), (C4, list(range(32))),
                                        (PROD, list(range(32)) + [511, 1023]), (C4K, list(range(32)))],
                         ids=["C2", "C3", "C4", "PROD", "C4K"])
def test_baseline_config_full_size(engine, coracle, cfg, sample):
    """BASELINE configs[1] (C2, 6.55 GB), configs[2] (C3, 64 GiB) and configs[3] at N = 1 (C4,
    10.24 GB), and the reference's default shapes at B = 1000 (PROD: 100M 8-byte timestamps, the
    rec8 record-space digest; C4K: C4 at B = 1000, the register-window digest): every digest, size,
    item count and root of every partition, standalone and fused; the sampled partitions equal the
    C oracle's build of host-regenerated records, nodes included."""
    from mydatastore_amd.workload import make_workload
    n_keys, P, V, B, mode = cfg
    w = make_workload(engine, n_partitions=P, n_buckets=B, value_len=V, part_mode=mode,
                      keys_per_partition=-(-n_keys // P), n_keys=n_keys)
    exp_dig, exp_size = _torch_digests(w)
    values, seg, n, _ = host_sample(coracle, n_keys, P, V, B, mode, sample)
    ref = coracle.build(values, seg, n, B, V, threads=16)
    del values
    assert np.array_equal(w.partition_ids, np.arange(P))  # N = 1: local slot == partition id
    for tag, o in _builds(engine, w):
        _check_full(o, w, exp_dig, exp_size, coracle, tag)
        sel ={k: v.reshape(P, -1)[sample].reshape(-1) for k, v in o.items()}
        _check_sample(sel, w, ref, n, tag)


def test_c5_anti_entropy_diff_and_extract_full_size(engine, coracle):
    """BASELINE configs[4] (C5) at C4 size: replica B = A with the first record of bucket
    (p * 37) % 64 of every partition changed. Both replicas built (standalone and fused), device
    DFS diff of every partition == exactly that bucket, and the out-of-sync range extract of B
    returns exactly that bucket's records of replica B, in partition order, with their bytes.
    The C oracle's builds and diffs of 32 host-regenerated partitions agree."""
    import torch
    from mydatastore_amd.workload import Workload, make_workload, perturb_replica
    import mydatastore_amd as mde
    n_keys, P, V, B, mode = C4
    w = make_workload(engine, n_partitions=P, n_buckets=B, value_len=V, part_mode=mode, n_keys=n_keys)
    dev = w.values.device
    vb, touched = perturb_replica(w)
    assert len(touched) == P  # every partition's perturbed bucket holds records at this size
    wb = Workload(engine, vb, w.seg_rec, P, B, w.n_records, V, w.partition_ids)
    a, b = w.build(), wb.build()
    # the fused shape the bench times: A and B alternate on one pipelined context
    sa, sb = w._outs(), wb._outs()
    engine.build_pipelined_async(w.rec, sa[1])
    engine.build_pipelined_async(wb.rec, sb[1])
    engine.build_pipeline_drain_async()
    engine.synchronize()
    for k in ("digest", "size", "items", "root", "nodes"):
        assert torch.equal(sa[0][k], a[k]) and torch.equal(sb[0][k], b[k]), k
    # independent digests of replica B
    exp_dig, exp_size = _torch_digests(wb)
    _check_full(b, wb, exp_dig, exp_size, coracle, "replica B")

    cap = mde.diff_capacity(B, B)
    ids = torch.full((P * cap,), -7, dtype=torch.int32, device=dev)
    cnt = torch.zeros(P, dtype=torch.int32, device=dev)
    engine.diff_async(P, B, a["digest"], a["nodes"], B, b["digest"], b["nodes"], ids, cap, cnt)
    rec_cap = w.n_records // 8
    part_off = torch.zeros(P + 1, dtype=torch.int64, device=dev)
    out_rec = torch.zeros(rec_cap, dtype=torch.int64, device=dev)
    out_vals = torch.zeros(rec_cap * V, dtype=torch.uint8, device=dev)
    out_voff = torch.zeros(rec_cap + 1, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    engine.extract_async(wb.rec, ids, cap, cnt, part_off, out_rec, rec_cap, out_vals, out_voff, rec_cap * V, status)
    engine.synchronize()
    cnt_h, ids_h = cnt.cpu().numpy(), ids.cpu().numpy().reshape(P, cap)
    for p in range(P):
        assert ids_h[p, :cnt_h[p]].tolist() == [touched[p]], p
    # expected extract: the touched bucket's record range of each partition, in partition order
    seg = w.seg_rec.cpu().numpy()
    want = np.concatenate([np.arange(seg[p * B + touched[p]], seg[p * B + touched[p] + 1]) for p in range(P)])
    assert int(status.item()) == 0
    po = part_off.cpu().numpy()
    assert po[-1] == want.size
    assert np.array_equal(np.diff(po), [seg[p * B + touched[p] + 1] - seg[p * B + touched[p]] for p in range(P)])
    n = want.size
    assert np.array_equal(out_rec[:n].cpu().numpy(), want)
    assert torch.equal(out_voff[:n + 1], torch.arange(n + 1, device=dev, dtype=torch.int64) * V)
    src = vb.view(-1, V)[torch.from_numpy(want).to(dev)]
    assert torch.equal(out_vals[:n * V].view(n, V), src)

    # the C oracle on 32 host-regenerated partitions: builds of A and B, and their DFS diffs
    sample = list(range(32))
    values, seg_s, ns, _ = host_sample(coracle, n_keys, P, V, B, mode, sample)
    vb_s, touched_s = perturb_first_record(values, seg_s, V, B, sample)
    assert touched_s == {i: touched[i] for i in sample}
    ra = coracle.build(values, seg_s, ns, B, V, threads=16)
    rb = coracle.build(vb_s, seg_s, ns, B, V, threads=16)
    _check_sample(a, w, ra, ns, "oracle A")
    _check_sample(b, wb, rb, ns, "oracle B")
    for i in sample:
        assert coracle.diff(ra["digest"][i * B:(i + 1) * B], rb["digest"][i * B:(i + 1) * B]) == [touched[i]]
