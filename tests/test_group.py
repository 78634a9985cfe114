"""Device groups (include/mde.h mde_group_*, csrc/group.cpp): one process driving the GPUs of a
node, partition p on device p % G, the roots all-gathered by RCCL (or device copies when a device
is listed twice) -- the in-node analogue of the reference's partition sharding over nodes
(hashring/hashring.go:126-154). On the one-GPU box a group lists device 0
once (RCCL, one rank) or several times (several contexts, copy gather): the sharding, rebasing,
slab layout and concurrent shard code are the ones an 8-GPU node runs. Plus two real processes
(gloo ranks sharing the GPU) running the engine on their shards."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT
from tests.datasets import MODES, synth_arrays


def _roots(out, P):
    return [out["root"][32 * p:32 * (p + 1)].tobytes().hex() for p in range(P)]


def _node_shas(out, P, B):
    import hashlib
    import mydatastore_amd as mde
    ni = mde.tree_internal_nodes(B) * 32
    return [hashlib.sha256(out["nodes"][ni * p:ni * (p + 1)].tobytes()).hexdigest() for p in range(P)]


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("streamed", [False, True], ids=["direct", "streamed"])
def test_multi_build_group(golden, coracle, devices, streamed):
    """mde_multi_build (partition p on device p % G, per-partition copies, RCCL or copy root
    gather) and mde_multi_build_streamed (the same placement, each device's partitions streamed
    through its two-slot ring, 4 KiB chunks) equal the golden single builds, layouts A and B,
    nodes included."""
    import mydatastore_amd as mde
    g = mde.Group(devices)
    assert len(g) == len(devices)
    assert g.gather_kind == ("rccl all_gather" if len(devices) == 1 else "device copies (a device listed twice)")
    kw = {"streamed": True, "chunk_bytes": 4096} if streamed else {}
    for case in golden("synth_cases.json"):
        values, voff, stride, seg = synth_arrays(case, coracle)
        P, B = case["P"], case["B"]
        out = g.build(values, P, B, stride, voff, seg_rec=seg, **kw)
        assert out["digest"].tolist() == case["digest"], case["name"]
        assert out["size"].tolist() == case["size"], case["name"]
        assert out["items"].tolist() == case["items"], case["name"]
        assert _roots(out, P) == case["root"], case["name"]
        assert _node_shas(out, P, B) == case["nodes_sha256"], case["name"]
        if not streamed:  # digest-only over the group: no tree, no gather
            d = g.build(values, P, B, stride, voff, seg_rec=seg, want_tree=False)
            assert d["digest"].tolist() == case["digest"] and d["root"] is None, case["name"]
        if case["var_len"]:
            continue
        n, V = case["n"], case["value_len"]
        gids = np.arange(n, dtype=np.uint64)
        part, bk = coracle.synth_tags(gids, P, B, MODES[case["part_mode"]], case["keys_per_partition"])
        order = np.argsort(part, kind="stable")
        part_rec = np.zeros(P + 1, np.uint64)
        np.cumsum(np.bincount(part, minlength=P), out=part_rec[1:])
        vb = coracle.synth_values(gids[order], V, case["seed"])
        ob = g.build(vb, P, B, V, part_rec=part_rec, bucket_tag=bk[order].astype(np.uint16), **kw)
        assert ob["digest"].tolist() == case["digest"], case["name"]
        assert _roots(ob, P) == case["root"], case["name"]
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["a", "b", "var"])
def test_every_group_entry_point_places_partition_p_on_member_p_mod_g(engine, layout):
    """One placement for the whole group API: mde_multi_build,
    mde_multi_build_streamed (several chunks per member) and the device-resident calls (a shard i
    built from partitions i, i + G, ...) all build partition p on member p % G. Observed through
    each member context's work accounting (mde_ctx_stats): the partitions and value bytes it built
    equal those of partitions p % G == i, on an arena whose partitions all differ in size."""
    import torch
    import mydatastore_amd as mde
    from mydatastore_amd.workload import make_workload
    G, P, B = 3, 11, 16
    rng = np.random.default_rng(5)
    counts = rng.integers(0, 40, P * B)
    counts[::7] = 0
    seg = np.zeros(P * B + 1, np.uint64)
    seg[1:] = np.cumsum(counts)
    n = int(seg[-1])
    V = 8
    voff = None
    if layout == "var":
        lens = rng.integers(0, 30, n)
        voff = np.zeros(n + 1, np.uint64)
        voff[1:] = np.cumsum(lens)
        values = rng.integers(0, 256, int(voff[-1]), dtype=np.uint8)
        V = 0
    else:
        values = rng.integers(0, 256, n * V, dtype=np.uint8)
    pos = (lambda r: int(voff[r])) if voff is not None else (lambda r: r * V)
    part_bytes = [pos(int(seg[(p + 1) * B])) - pos(int(seg[p * B])) for p in range(P)]
    want = [(sum(1 for p in range(P) if p % G == i), sum(part_bytes[p] for p in range(P) if p % G == i))
            for i in range(G)]
    assert len({b for _, b in want}) == G  # the members' byte totals tell the placements apart
    g = mde.Group([0] * G)

    def delta(fn):
        before = [g.ctx_stats(i) for i in range(G)]
        fn()
        after = [g.ctx_stats(i) for i in range(G)]
        return [(a["partitions"] - b["partitions"], a["value_bytes"] - b["value_bytes"]) for a, b in zip(after, before)]

    if layout == "b":
        part_rec = seg[::B].copy()
        tags = np.repeat(np.tile(np.arange(B, dtype=np.uint16), P), counts)
        kw = dict(part_rec=part_rec, bucket_tag=tags)
    else:
        kw = dict(value_off=voff, seg_rec=seg)
    ref = g.build(values, P, B, V, **kw)
    assert delta(lambda: g.build(values, P, B, V, **kw)) == want
    st = delta(lambda: g.build(values, P, B, V, streamed=True, chunk_bytes=256, **kw))
    assert st == want, (st, want)
    got = g.build(values, P, B, V, streamed=True, chunk_bytes=256, **kw)
    for k in ("digest", "size", "items", "root", "nodes"):
        assert np.array_equal(got[k], ref[k]), k
    if layout == "a":  # device-resident: shard i = partitions i, i + G, ... (make_workload's split)
        shards = [make_workload(engine, n_partitions=P, n_buckets=B, value_len=8, part_mode="mod", n_keys=3000,
                                rank=i, world=G) for i in range(G)]
        for i, w in enumerate(shards):
            assert list(w.partition_ids) == list(range(i, P, G)) and w.n_partitions == g.partitions(P, i)
        outs = [w._outs() for w in shards]
        d = delta(lambda: (g.build_async([w.rec for w in shards], [o[1] for o in outs]), g.synchronize()))
        assert d == [(len(range(i, P, G)), shards[i].value_bytes) for i in range(G)]
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("B", [64, 1000])
def test_group_device_resident_build_and_gather(engine, devices, B):
    """The path bench.py times at N > 1: every device's shard (partition p on device p % G,
    generated on the device) built by mde_group_build_async and by a run of pipelined builds, then
    ONE all-gather of the fixed-size root slabs: every device receives the same slabs, and they
    assemble to exactly the roots of one engine build of the whole workload."""
    import torch
    import mydatastore_amd as mde
    from mydatastore_amd.workload import make_workload
    G, P, V, n = len(devices), 100, 64, 300_000
    g = mde.Group(devices)
    dev = torch.device("cuda:0")
    shards = [make_workload(engine, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n,
                            rank=i, world=G) for i in range(G)]
    for i, w in enumerate(shards):
        assert w.n_partitions == g.partitions(P, i)
    whole = make_workload(engine, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n)
    want = whole.build()["root"].cpu().numpy().reshape(P, 32)
    slab = -(-P // G)
    for pipelined in (False, True):
        outs = [w._outs() for w in shards]
        g.build_async([w.rec for w in shards], [o[1] for o in outs], pipelined=pipelined)
        if pipelined:  # the second build of the run carries the first one's trees
            outs2 = [w._outs() for w in shards]
            g.build_async([w.rec for w in shards], [o[1] for o in outs2], pipelined=True)
            g.drain_async()
        g.synchronize()
        send = [torch.zeros(slab * 32, dtype=torch.uint8, device=dev) for _ in range(G)]
        recv = [torch.zeros(G * slab * 32, dtype=torch.uint8, device=dev) for _ in range(G)]
        for i in range(G):
            send[i][:shards[i].n_partitions * 32].copy_(outs[i][0]["root"])
        torch.cuda.synchronize(dev)
        g.gather_async(send, recv, slab * 32)
        g.synchronize()
        got = recv[0].cpu().numpy().reshape(G, slab, 32)
        for i in range(1, G):
            assert torch.equal(recv[i], recv[0])
        assembled = np.zeros((P, 32), np.uint8)
        for r in range(G):
            pids = shards[r].partition_ids
            assembled[pids] = got[r, :len(pids)]
        assert np.array_equal(assembled, want), pipelined
    g.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_two_gloo_ranks_run_the_engine():
    """Two fresh processes (torch.distributed.run, gloo, both on cuda:0) each build their shard
    with the ENGINE (not the oracle); the gathered roots equal one process's engine build of the
    whole workload."""
    env = {**os.environ, "MASTER_ADDR": "127.0.0.1"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(ROOT / "tests" / "dist_engine_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["world"] == 2
    assert d["gathered_roots_equal_single_process"] and d["rank0_digests_equal_single_process"], d
    assert d["engine"].endswith("libmde.so")


def test_group_symbols_and_cpu_behaviour():
    """CPU: the group entry points exist; without a GPU mde_group_create fails loudly."""
    import ctypes as C
    import torch
    import mydatastore_amd as mde
    lib = mde.load_library()
    for name in ("mde_group_gather_kind", "mde_group_partitions", "mde_group_build_async",
                 "mde_group_gather_async", "mde_device_count"):
        assert hasattr(lib, name)
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert lib.mde_device_count() == 0
    devs = (C.c_int * 1)(0)
    h = C.c_void_p()
    assert lib.mde_group_create(devs, 1, C.byref(h)) == mde.MDE_E_DEVICE and not h.value


@pytest.mark.gpu
@pytest.mark.parametrize("gpus,config", [(1, "c4"), (2, "c4"), (8, "c4"), (1, "c5"), (8, "c5")])
def test_bench_group_mode(gpus, config):
    """bench.py's N-GPU path (--engine group) end to end on the box: one process, the shards of
    BASELINE config 4 (or 5: both replicas, diff, extract) over `gpus` group members (GPU 0 listed
    `gpus` times: --rehearse), pipelined builds and side-stream root gathers; its parity block
    (gathered slabs, the C-oracle sample of shard 0; C5: every gathered diff count and shard 0's
    diff and extract) is all true, and the line carries the per-build gather cost and the host
    enqueue time the >= 6x target depends on."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--engine", "group", "--gpus", str(gpus), "--steps", "9",
           "--warmup", "2", "--config", config] + (["--rehearse"] if gpus > 1 else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["parity"]["all_ranks_ok"], d["parity"]
    assert d["config"]["engine"] == "group" and d["n_gpus"] == gpus
    assert ("rccl" in d["config"]["root_gather"]) == (gpus == 1)
    assert d["host_timing"]["enqueue_ms_per_step"] > 0
    if config == "c4":
        assert d["root_gather_per_build"]["gathered_roots_match_after_run"]
        assert d["root_gather_per_build"]["bare_gather_ms"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("overlapped", [False, True], ids=["in_stream", "overlapped"])
def test_gather_send_slab_rewritten_right_after_the_gather(overlapped):
    """The exchange step's stream-order contract with the copy gather (a device listed three
    times): work enqueued on a context stream after the gather -- here each device rewriting its
    own send slab at once -- must not change what the other devices receive. The in-stream gather
    makes every context stream wait for every device's copies; the overlapped one does once the
    caller waits on its ticket (mde_group_gather_wait_async) before the rewrite."""
    import torch
    import mydatastore_amd as mde
    G, nbytes = 3, 64 << 20
    g = mde.Group([0] * G)
    dev = torch.device("cuda:0")
    lib = mde.load_library()
    streams = [torch.cuda.ExternalStream(lib.mde_get_stream(g.ctx(i)), device=dev) for i in range(G)]
    send = [torch.full((nbytes,), i + 1, dtype=torch.uint8, device=dev) for i in range(G)]
    recv = [torch.zeros(G * nbytes, dtype=torch.uint8, device=dev) for _ in range(G)]
    torch.cuda.synchronize(dev)
    for rep in range(3):
        if overlapped:
            t = g.gather_overlapped_async(send, recv, nbytes)
            g.gather_wait_async(t)
        else:
            g.gather_async(send, recv, nbytes)
        for i in range(G):  # the rewrite, in stream order right after the gather
            with torch.cuda.stream(streams[i]):
                send[i].fill_(0xEE)
        g.synchronize()
        for i in range(G):
            got = recv[i].view(G, nbytes)
            for r in range(G):
                assert bool((got[r] == r + 1 + 16 * rep).all()), (rep, i, r)
        for i in range(G):
            send[i].fill_(i + 1 + 16 * (rep + 1))
            recv[i].zero_()
        torch.cuda.synchronize(dev)
    g.close()


def _c5_single(engine, P, B, V, n):
    """BASELINE config 5 in one engine: replicas A and B of the whole workload, diff + extract."""
    import torch
    import mydatastore_amd as mde
    from mydatastore_amd.workload import Workload, make_workload, perturb_replica
    w = make_workload(engine, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n)
    vb, touched = perturb_replica(w)
    wb = Workload(engine, vb, w.seg_rec, P, B, w.n_records, V, w.partition_ids)
    oa, ob = w.build(), wb.build()
    cap = mde.diff_capacity(B, B)
    dev = w.values.device
    ids = torch.zeros(P * cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(P, dtype=torch.int32, device=dev)
    engine.diff_async(P, B, oa["digest"], oa["nodes"], B, ob["digest"], ob["nodes"], ids, cap, cnt)
    rec_cap = max(w.n_records, 1024)  # B = 1 or 2 extracts all or half of the records
    part_off = torch.zeros(P + 1, dtype=torch.int64, device=dev)
    out_rec = torch.zeros(rec_cap, dtype=torch.int64, device=dev)
    out_vals = torch.zeros(rec_cap * V, dtype=torch.uint8, device=dev)
    out_voff = torch.zeros(rec_cap + 1, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    engine.extract_async(wb.rec, ids, cap, cnt, part_off, out_rec, rec_cap, out_vals, out_voff, rec_cap * V, status)
    engine.synchronize()
    po = part_off.cpu().numpy().astype(np.int64)
    vals = out_vals.cpu().numpy()
    per_part = [vals[po[p] * V:po[p + 1] * V].tobytes() for p in range(P)]
    c = cnt.cpu().numpy()
    idl = ids.cpu().numpy().reshape(P, cap)
    return {"roots_a": oa["root"].cpu().numpy().reshape(P, 32), "roots_b": ob["root"].cpu().numpy().reshape(P, 32),
            "digest_a": oa["digest"].cpu().numpy().reshape(P, B), "digest_b": ob["digest"].cpu().numpy().reshape(P, B),
            "counts": c, "ids": [idl[p, :c[p]].tolist() for p in range(P)], "extract": per_part,
            "status": int(status.item()), "touched": touched}


@pytest.mark.gpu
@pytest.mark.parametrize("G,P,B,V,n", [(1, 48, 64, 64, 120_000), (2, 48, 64, 64, 120_000), (8, 48, 64, 64, 120_000),
                                       (8, 5, 64, 32, 20_000), (3, 37, 999, 8, 90_000), (5, 64, 130, 24, 70_000)],
                         ids=["G1", "G2", "G8", "G8-P5-members-without-partitions", "G3-odd-B999-8B", "G5-B130"])
def test_group_c5_diff_extract_and_gather(engine, G, P, B, V, n):
    """BASELINE config 5 on the mde_group path (the one the Go shim's process reaches): each
    device builds both replicas of its partitions (pipelined, as bench.py times it), diffs them and
    extracts replica B's records of the differing buckets on the device (mde_group_diff_async,
    mde_group_extract_async), and the [A roots | B roots | diff counts | diff ids] slabs (the
    diff writes its counts and id lists into the slab itself) are all-gathered on the side
    streams (mde_group_gather_overlapped_async). The gathered slabs, every shard's diff ids and
    extracted bytes equal the single-engine C5 result; the diff of every partition is the
    oracle's DFS diff: its perturbed bucket, once per odd level on the bucket's path. Shapes:
    1/2/8 members, more members than partitions (members with nothing to build still take part
    in the gather), odd B with 8-byte values, B = 130."""
    _check_group_c5(engine, G, P, B, V, n)


def _random_c5_shapes(k, seed=20261018):
    """Seeded random C5 shapes for the group: member counts 1-8, partition counts 1-79 (members
    without partitions when G > P), B from 1 to 333 (odd levels: DFS duplicates), values of
    1-33 bytes (the 8-byte record scan among them), a few to ~40 records per bucket."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        G, P = int(rng.integers(1, 9)), int(rng.integers(1, 80))
        B = int(rng.choice([1, 2, 3, 5, 31, 64, 65, 130, 333]))
        V = int(rng.choice([1, 3, 8, 8, 16, 33]))
        n = max(1, min(200_000, P * B * int(rng.integers(1, 40))))
        out.append((G, P, B, V, n))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("G,P,B,V,n", _random_c5_shapes(8))
def test_group_c5_random_shapes(engine, G, P, B, V, n):
    """The group C5 check of test_group_c5_diff_extract_and_gather over seeded random shapes."""
    _check_group_c5(engine, G, P, B, V, n)


def _check_group_c5(engine, G, P, B, V, n):
    import torch
    import mydatastore_amd as mde
    from mydatastore_amd.workload import Workload, make_workload, perturb_replica
    ref = _c5_single(engine, P, B, V, n)
    assert ref["status"] == 0
    for p in range(P):  # the DFS diff of the perturbed bucket: repeated once per odd level on its
        # path (the reference visits a self-paired node's child twice), nothing for the others
        if p in ref["touched"]:
            assert ref["ids"][p] == O.diff_from_digests(ref["digest_a"][p], ref["digest_b"][p])
            assert set(ref["ids"][p]) == {ref["touched"][p]}
        else:
            assert ref["ids"][p] == [] and np.array_equal(ref["digest_a"][p], ref["digest_b"][p])
    g = mde.Group([0] * G)
    dev = torch.device("cuda:0")
    slab = -(-P // G)
    cap = mde.diff_capacity(B, B)
    shards, repl, outs, args_d, args_x, x, keep = [], [], [], [], [], [], []
    width = 68 + 4 * cap
    send = [torch.zeros(slab * width, dtype=torch.uint8, device=dev) for _ in range(G)]
    recv = [torch.zeros(G * slab * width, dtype=torch.uint8, device=dev) for _ in range(G)]
    for i in range(G):
        w = make_workload(engine, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n, rank=i, world=G)
        vb, _ = perturb_replica(w)
        wb = Workload(engine, vb, w.seg_rec, w.n_partitions, B, w.n_records, V, w.partition_ids)
        Pl = w.n_partitions
        oa, ob = w._outs()[0], wb._outs()[0]
        keep.append((oa, ob))  # the output tensors live as long as the group's launches
        base = send[i].data_ptr()
        to_a = mde.TreeOut(oa["digest"].data_ptr(), oa["size"].data_ptr(), oa["items"].data_ptr(), base,
                           oa["nodes"].data_ptr())
        to_b = mde.TreeOut(ob["digest"].data_ptr(), ob["size"].data_ptr(), ob["items"].data_ptr(), base + slab * 32,
                           ob["nodes"].data_ptr())
        ids_ptr = base + slab * 68  # the diff id lists land in the send slab too
        rec_cap = max(w.n_records, 1024)  # B = 1 or 2 extracts all or half of the records
        t = {"part_off": torch.zeros(Pl + 1, dtype=torch.int64, device=dev),
             "out_rec": torch.zeros(rec_cap, dtype=torch.int64, device=dev),
             "out_vals": torch.zeros(rec_cap * V, dtype=torch.uint8, device=dev),
             "out_voff": torch.zeros(rec_cap + 1, dtype=torch.int64, device=dev),
             "status": torch.zeros(1, dtype=torch.int32, device=dev)}
        counts_ptr = base + slab * 64  # the diff counts land in the send slab itself
        args_d.append(mde.DiffArgs(Pl, B, B, oa["digest"].data_ptr(), oa["nodes"].data_ptr(), ob["digest"].data_ptr(),
                                   ob["nodes"].data_ptr(), ids_ptr, cap, counts_ptr))
        args_x.append(mde.ExtractArgs(ids_ptr, cap, counts_ptr, t["part_off"].data_ptr(),
                                      t["out_rec"].data_ptr(), rec_cap, t["out_vals"].data_ptr(),
                                      t["out_voff"].data_ptr(), rec_cap * V, t["status"].data_ptr()))
        shards.append(w)
        repl.append(wb)
        outs.append((to_a, to_b))
        x.append(t)
    torch.cuda.synchronize(dev)
    # replica A then replica B, pipelined: B's launch completes A's trees, the drain B's
    g.build_async([w.rec for w in shards], [o[0] for o in outs], pipelined=True)
    g.build_async([w.rec for w in repl], [o[1] for o in outs], pipelined=True)
    g.drain_async()
    g.diff_async(args_d)
    g.extract_async([w.rec for w in repl], args_x)
    ticket = g.gather_overlapped_async(send, recv, slab * width)
    g.gather_wait_async(ticket)
    g.synchronize()
    for i in range(1, G):
        assert torch.equal(recv[i], recv[0])
    got = recv[0].cpu().numpy().reshape(G, slab * width)
    for r in range(G):
        pids = shards[r].partition_ids
        k = len(pids)
        assert np.array_equal(got[r, :k * 32].reshape(k, 32), ref["roots_a"][pids]), r
        assert np.array_equal(got[r, slab * 32:slab * 32 + k * 32].reshape(k, 32), ref["roots_b"][pids]), r
        assert np.array_equal(got[r, slab * 64:slab * 64 + k * 4].view(np.int32), ref["counts"][pids]), r
        assert int(x[r]["status"].item()) == 0
        ids = got[r, slab * 68:slab * 68 + k * cap * 4].view(np.int32).reshape(k, cap)
        po = x[r]["part_off"].cpu().numpy().astype(np.int64)
        vals = x[r]["out_vals"].cpu().numpy()
        cnt = ref["counts"][pids]
        for j, p in enumerate(pids):
            assert ids[j, :cnt[j]].tolist() == ref["ids"][p], (r, p)
            assert vals[po[j] * V:po[j + 1] * V].tobytes() == ref["extract"][p], (r, p)
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c4", "c5"])
def test_bench_group_under_torchrun(config):
    """The driver's N-GPU invocation (`torch.distributed.run --nproc-per-node N bench.py --gpus N`):
    rank 0 drives the group, the other ranks only join its barriers -- the same number of them for
    every config (two around each timed run, one at the end), or a rank would wait forever. Two
    ranks, both shards on GPU 0 (--rehearse)."""
    env = {**os.environ, "MASTER_ADDR": "127.0.0.1"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "1", "--rehearse", "--config", config]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["parity"]["all_ranks_ok"] and d["launcher_ranks"] == 2 and d["config"]["engine"] == "group"
    assert (d["root_gather_per_build"] is not None) == (config == "c4")


@pytest.mark.gpu
def test_group_errors_name_the_failing_member(engine):
    """With one enqueue thread per member, a failure on one member still comes back as the call's
    error, naming that member; the other members' shares were enqueued and the group stays usable.
    An unknown gather ticket is MDE_E_INVAL."""
    import torch
    import mydatastore_amd as mde
    from mydatastore_amd.workload import make_workload
    G, P, B, V, n = 3, 30, 64, 32, 30_000
    g = mde.Group([0] * G)
    shards = [make_workload(engine, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n, rank=i,
                            world=G) for i in range(G)]
    outs = [w._outs() for w in shards]
    bad = mde.Records.from_buffer_copy(shards[2].rec)
    bad.n_buckets = 0  # rejected by mde_build_async on member 2
    with pytest.raises(mde.MdeError) as ei:
        g.build_async([shards[0].rec, shards[1].rec, bad], [o[1] for o in outs])
    assert ei.value.code == mde.MDE_E_INVAL and "member 2" in str(ei.value)
    g.synchronize()
    with pytest.raises(mde.MdeError) as ei:
        g.gather_wait_async(12345)
    assert ei.value.code == mde.MDE_E_INVAL
    g.build_async([w.rec for w in shards], [o[1] for o in outs])  # still usable
    g.synchronize()
    whole = make_workload(engine, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n)
    want = whole.build()["root"].cpu().numpy().reshape(P, 32)
    for i, w in enumerate(shards):
        assert np.array_equal(outs[i][0]["root"].cpu().numpy().reshape(-1, 32), want[w.partition_ids])
    g.close()
    torch.cuda.synchronize()


GROUP_CABI = ROOT / "tests" / "cpp" / "build" / "group_cabi"


def test_group_cabi_fails_loudly_without_gpu():
    """The plain-C driver of the multi-GPU path builds, and without a gfx950 device it stops at
    mde_device_list (there is no CPU fallback behind the ABI)."""
    import torch
    subprocess.run([sys.executable, "-m", "mydatastore_amd._build", "-q"], cwd=ROOT, check=True)
    assert GROUP_CABI.exists()
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([str(GROUP_CABI), "1000", "4", "64", "8", "2", "1"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no gfx950 device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("members,rehearse", [(1, 0), (3, 1), (8, 1)])
def test_group_cabi_parity(members, rehearse):
    """The multi-GPU path from plain C, no PyTorch (what one node process does with its GPUs): a
    reduced C4-shaped workload sharded p % G, pipelined group builds with the roots in the send
    slabs and one overlapped gather per build; the last build's gathered slabs hold every member's
    roots on every member, equal a standalone group build's, and member 0's roots are the tree of
    its digests. One GPU: 1 member over RCCL, 3 and 8 members rehearsed on it (device copies)."""
    import json
    r = subprocess.run([str(GROUP_CABI), "1000000", "256", "256", "64", "6", "2", str(members), str(rehearse)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert all(d["parity"].values()), d
    assert d["members"] == members and ("rccl" in d["gather"]) == (members == 1)


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c4", "c5"])
def test_bench_ranks_engine_under_torchrun(config):
    """The one-process-per-GPU path (`--engine ranks`) at two ranks, both on GPU 0 with the gloo
    gather (--rehearse): every parity gate holds, for C5 including the gathered diff counts and
    diff-id lists of every rank."""
    env = {**os.environ, "MASTER_ADDR": "127.0.0.1"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--rehearse", "--engine", "ranks", "--config", config,
           "--no-gather-per-build"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["parity"]["all_ranks_ok"], d["parity"]
    if config == "c5":
        assert d["parity"]["c5_gathered_diff_ids"] and d["parity"]["c5_gathered_diff_counts"]
