#!/usr/bin/env python3
"""Kernel micro-benchmarks (HIP events on the launch stream).

    python tools/microbench.py tree            # tree kernel vs partitions / buckets
    python tools/microbench.py digest          # digest kernel vs arena size (C4 shards)
    python tools/microbench.py verify          # mde_verify_epochs vs partitions (2 peers each)
    python tools/microbench.py decode          # mde_decode_epoch_tree_objects_async, B = 64 / 1000
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def timeit(fn, reps=20, warm=3):
    import torch
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def bench_tree(eng):
    import torch
    import mydatastore_amd as mde
    res = []
    for B in (64, 1000):
        for P in (1, 8, 128, 256, 1024, 4096):
            d = torch.randint(0, 999999, (P * B,), dtype=torch.int64, device="cuda")
            root = torch.zeros(P * 32, dtype=torch.uint8, device="cuda")
            nodes = torch.zeros(P * mde.tree_internal_nodes(B) * 32, dtype=torch.uint8, device="cuda")
            us = timeit(lambda: eng.tree_from_digests_async(P, B, d, root, nodes))
            res.append({"kernel": "tree", "B": B, "P": P, "us": round(us, 2)})
            print(json.dumps(res[-1]), flush=True)
    return res


def bench_digest(eng, worlds=(8, 4, 2, 1)):
    from mydatastore_amd.workload import make_workload
    res = []
    for world in worlds:
        w = make_workload(eng, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                          n_keys=10_000_000, rank=0, world=world)
        us = timeit(w.digest_async)
        ust = timeit(w.tree_async)
        usb = timeit(w.build_async)
        res.append({"kernel": "digest", "world": world, "bytes": w.value_bytes, "digest_us": round(us, 2),
                    "GBps": round(w.value_bytes / us / 1e3, 1), "tree_us": round(ust, 2),
                    "build_us": round(usb, 2)})
        print(json.dumps(res[-1]), flush=True)
        del w
    return res


def bench_sweep(eng, worlds=(1, 8), reps=3):
    """Interleaved A/B of digest variants x workgroups-per-CU in one process (same data, same
    clocks): median digest time per setting."""
    from mydatastore_amd.workload import make_workload
    settings = [(v, c) for v in range(7) for c in (0, 2, 3, 4)]
    res = []
    for world in worlds:
        w = make_workload(eng, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                          n_keys=10_000_000, rank=0, world=world)
        times = {s: [] for s in settings}
        for _ in range(reps):
            for v, c in settings:
                eng.set_tuning(v, c)
                times[(v, c)].append(timeit(w.digest_async, reps=10, warm=2))
        eng.set_tuning(-1, -1)
        for (v, c), t in times.items():
            med = float(np.median(t))
            res.append({"world": world, "variant": v, "cap": c, "digest_us": round(med, 2),
                        "GBps": round(w.value_bytes / med / 1e3, 1)})
        best = sorted([r for r in res if r["world"] == world], key=lambda r: r["digest_us"])[:6]
        for r in best:
            print(json.dumps(r), flush=True)
        del w
    return res


def bench_ab(eng, variants, worlds=(1, 8), reps=5, cap=2):
    """Interleaved A/B of digest variants at one workgroups-per-CU cap (same data, same clocks)."""
    from mydatastore_amd.workload import make_workload
    res = []
    for world in worlds:
        w = make_workload(eng, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                          n_keys=10_000_000, rank=0, world=world)
        ref = None
        times = {v: [] for v in variants}
        for _ in range(reps):
            for v in variants:
                eng.set_tuning(v, cap)
                times[v].append(timeit(w.digest_async, reps=10, warm=2))
                o = w.build()
                if ref is None:
                    ref = o["root"].cpu()
                assert bool((o["root"].cpu() == ref).all()), f"variant {v} roots differ"
        eng.set_tuning(-1, -1)
        for v, t in times.items():
            med = float(np.median(t))
            res.append({"world": world, "variant": v, "cap": cap, "digest_us": round(med, 2),
                        "GBps": round(w.value_bytes / med / 1e3, 1)})
            print(json.dumps(res[-1]), flush=True)
        del w
    return res


# Workload shapes for the digest probes (make_workload arguments over the C4 defaults).
SHAPES = {"c4": dict(n_partitions=1024, n_keys=10_000_000, part_mode="mod", world=1),
              "c4/8": dict(n_partitions=1024, n_keys=10_000_000, part_mode="mod", world=8),
              "c3": dict(n_partitions=64, n_keys=64_000_000, part_mode="block", world=1),
              "c4b": dict(n_partitions=1024, n_keys=10_000_000, part_mode="mod", world=1, layout="b"),
              "c4b/8": dict(n_partitions=1024, n_keys=10_000_000, part_mode="mod", world=8, layout="b"),
              # the reference's default PartitionBuckets (config/default-config.yaml:8)
              "c4k": dict(n_partitions=1024, n_keys=10_000_000, part_mode="mod", world=1, n_buckets=1000),
              "c4k/8": dict(n_partitions=1024, n_keys=10_000_000, part_mode="mod", world=8, n_buckets=1000),
              # production values: the 8-byte LE write timestamp (main/manager.go:816)
              "ts8": dict(n_partitions=1024, n_keys=100_000_000, part_mode="mod", world=1, value_len=8),
              "ts8k": dict(n_partitions=1024, n_keys=100_000_000, part_mode="mod", world=1, value_len=8,
                           n_buckets=1000),
              "c4bk": dict(n_partitions=1024, n_keys=10_000_000, part_mode="mod", world=1, layout="b",
                           n_buckets=1000),
              "ts8bk": dict(n_partitions=1024, n_keys=100_000_000, part_mode="mod", world=1, value_len=8,
                            n_buckets=1000, layout="b"),
              "v64k": dict(n_partitions=1024, n_keys=20_000_000, part_mode="mod", world=1, value_len=64,
                           n_buckets=1000)}


def apply_setting(eng, p):
    """Digest variant / piece setting by name (see bench_pieces); a suffix "@N" caps the resident
    digest workgroups per CU at N."""
    cap = -1
    if "@" in p:
        p, c = p.split("@")
        cap = int(c)
    v, rest = (11 if p == "x" else -1), p
    if p.startswith("v"):
        num = "".join(ch for ch in p[1:] if ch.isdigit())
        v, rest = int(num), p[1 + len(num):].lstrip("_")
    elif p not in ("d", "x"):
        v = 12
    eng.set_tuning(v, cap)
    eng.set_digest_piece_bytes({"d": -1, "x": 0}[rest] if rest in ("d", "x") else int(rest))


def bench_pieces(eng, pieces, shapes=("c4", "c4/8", "c3"), reps=5):
    """Interleaved A/B of the layout-A digest work split: the defaults ("d", automatic pieces),
    the default variant with one contiguous range per wave ("x") and the interleaved-pieces
    variant at N-byte pieces (0 = its loop with one piece per wave). Per setting: the standalone
    digest kernel and a run of fused pipelined builds (build_step_kernel), median over reps;
    every setting's roots must equal the first setting's."""
    import torch
    from mydatastore_amd.workload import make_workload
    res = []
    for shape in shapes:
        w = make_workload(eng, **{"n_buckets": 64, "value_len": 1024, "rank": 0, **SHAPES[shape]})
        sets = [w._outs() for _ in range(2)]
        n_steps = 10

        def fused(n=n_steps):
            for i in range(n):
                eng.build_pipelined_async(w.rec, sets[i % 2][1])
            eng.build_pipeline_drain_async()

        ref = None
        td = {p: [] for p in pieces}
        tf = {p: [] for p in pieces}
        ts = {p: [] for p in pieces}  # steady state: (2n builds - n builds) / n, the drain cancels
        tt = {p: [] for p in pieces}
        for _ in range(reps):
            for p in pieces:
                # "d": the defaults (automatic variant and pieces); "x": variant 11 (round 1's
                # default) with one range per wave; a number: the interleaved-pieces variant at that piece size; "v13d",
                # "v13x", "v14_1048576": variant 13 / 14 with the same piece settings
                apply_setting(eng, p)
                td[p].append(timeit(w.digest_async, reps=10, warm=2))
                t1 = timeit(fused, reps=1, warm=1)
                tf[p].append(t1 / n_steps)
                # both runs warmed back to back: a run that starts on an idle GPU pays its clock ramp
                # (the tree-bound steps show it, the HBM-bound stream does not)
                ts[p].append((timeit(lambda: fused(2 * n_steps), reps=1, warm=1) - t1) / n_steps)
                tt[p].append(timeit(w.tree_async, reps=5, warm=1))
                o = w.build()
                if ref is None:
                    ref = o["root"].cpu()
                assert bool((o["root"].cpu() == ref).all()), f"pieces {p}: roots differ"
        eng.set_digest_piece_bytes(-1)
        eng.set_tuning(-1, -1)
        for p in pieces:
            md, mf = float(np.median(td[p])), float(np.median(tf[p]))
            res.append({"shape": shape, "piece_bytes": p, "bytes": w.value_bytes, "digest_us": round(md, 2),
                        "digest_GBps": round(w.value_bytes / md / 1e3, 1), "fused_us_per_build": round(mf, 2),
                        "fused_GBps": round(w.value_bytes / mf / 1e3, 1),
                        "fused_steady_us": round(float(np.median(ts[p])), 2),
                        "tree_us": round(float(np.median(tt[p])), 2)})
            print(json.dumps(res[-1]), flush=True)
        del w, sets
        torch.cuda.empty_cache()
    return res


def bench_digest_only(eng, shape, reps=5, setting="d"):
    """The digest kernel alone on one workload shape, `reps` launches (for rocprofv3 PMC passes: no
    other kernels between the workload build and the launches but its own); `setting` as in
    bench_pieces (default: the automatic choice)."""
    from mydatastore_amd.workload import make_workload
    w = make_workload(eng, **{"n_buckets": 64, "value_len": 1024, "rank": 0, **SHAPES[shape]})
    apply_setting(eng, setting)
    us = timeit(w.digest_async, reps=reps, warm=1)
    r = {"shape": shape, "setting": setting, "bytes": w.value_bytes, "digest_us": round(us, 2),
         "digest_GBps": round(w.value_bytes / us / 1e3, 1)}
    print(json.dumps(r), flush=True)
    return r


def bench_fused_only(eng, shape, reps=5):
    """`reps` fused pipelined builds (build_step_kernel / tagged_step_kernel) of one workload shape
    and the drain, nothing else after the workload build (for rocprofv3 PMC passes)."""
    from mydatastore_amd.workload import make_workload
    w = make_workload(eng, **{"n_buckets": 64, "value_len": 1024, "rank": 0, **SHAPES[shape]})
    sets = [w._outs() for _ in range(2)]

    def run():
        for i in range(reps):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        eng.build_pipeline_drain_async()

    us = timeit(run, reps=1, warm=1) / reps
    r = {"shape": shape, "bytes": w.value_bytes, "fused_us_per_build": round(us, 2),
         "fused_GBps": round(w.value_bytes / us / 1e3, 1)}
    print(json.dumps(r), flush=True)
    return r


def bench_step_stamps(eng, shape, reps=8):
    """Probe library only (-DMDE_STEP_STAMPS): per fused build step, when the first / last tree
    wave and the first / last streaming wave started and ended (s_memrealtime, 100 MHz), relative
    to the first streaming wave's start, in us."""
    import ctypes as C
    import torch
    from mydatastore_amd.workload import make_workload
    fn = eng.lib.mde_probe_step_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    buf = (C.c_ulonglong * 4)()
    w = make_workload(eng, **{"n_buckets": 64, "value_len": 1024, "rank": 0, **SHAPES[shape]})
    sets = [w._outs() for _ in range(2)]
    rows = []
    for i in range(reps + 2):
        torch.cuda.synchronize()
        fn(buf, 1)
        eng.build_pipelined_async(w.rec, sets[i % 2][1])
        torch.cuda.synchronize()
        fn(buf, 0)
        t = list(buf)
        if i < 2:
            continue
        z = t[2]
        r = {"shape": shape, "tree_start_us": round((t[0] - z) / 100, 2), "tree_end_us": round((t[1] - z) / 100, 2),
             "stream_end_us": round((t[3] - z) / 100, 2)}
        rows.append(r)
        print(json.dumps(r), flush=True)
    eng.build_pipeline_drain_async()
    torch.cuda.synchronize()
    return rows


def bench_verify(eng, P=1024, B=64, R=2, mode=0):
    """VerifyEpoch decision step (mde_verify_epochs) for P partitions x R peer objects: peer 0
    agrees, peer 1 differs in one bucket. Device-resident call timed with HIP events; the
    synchronous host call (copies included) with the wall clock."""
    import time
    import torch
    from mydatastore_amd.workload import make_workload
    dev = torch.device("cuda:0")
    w = make_workload(eng, n_partitions=P, n_buckets=B, value_len=64, part_mode="mod", n_keys=P * 2000)
    out = w.build()
    dg = out["digest"].cpu().numpy().view(np.uint64)
    sz = out["size"].cpu().numpy()
    same = eng.encode_objects(B, dg, sz, partition=np.arange(P, dtype=np.int32), lower=5, upper=6)
    d2 = dg.copy()
    d2[::B] = (d2[::B] + 1) % 999999
    diff = eng.encode_objects(B, d2, sz, partition=np.arange(P, dtype=np.int32), lower=5, upper=6)
    peers = [[same[p], diff[p]][:R] for p in range(P)]
    flat = [o for row in peers for o in row]
    off = np.zeros(len(flat) + 1, np.int64)
    off[1:] = np.cumsum([len(o) for o in flat])
    blob = torch.from_numpy(np.frombuffer(b"".join(flat), dtype=np.uint8).copy()).to(dev)
    doff = torch.from_numpy(off).to(dev)
    stride = int(eng.lib.mde_epoch_tree_object_max_bytes(B))
    o = {"valid": torch.zeros(P, dtype=torch.uint8, device=dev), "vc": torch.zeros(P, dtype=torch.int32, device=dev),
         "ids": torch.zeros(P * B, dtype=torch.int32, device=dev), "dc": torch.zeros(P, dtype=torch.int32, device=dev),
         "st": torch.zeros(P * R, dtype=torch.int32, device=dev),
         "obj": torch.zeros(P * stride, dtype=torch.uint8, device=dev), "olen": torch.zeros(P, dtype=torch.int32, device=dev)}

    def dev_call():
        eng.verify_epochs_async(P, B, None, 5, out["digest"], out["size"], out["nodes"], R, blob, doff, 2,
                                o["valid"], o["vc"], o["ids"], o["dc"], o["st"], o["obj"], stride, o["olen"])

    eng.set_verify_mode(mode)
    us_dev = timeit(dev_call, reps=20, warm=3)
    assert int(o["vc"].sum()) == P and int(o["dc"].sum()) == P  # one agreeing peer, one differing bucket
    nodes = out["nodes"].cpu().numpy()
    eng.verify_epochs(B, dg, sz, nodes, peers, 2, 5)
    t0 = time.perf_counter()
    for _ in range(5):
        eng.verify_epochs(B, dg, sz, nodes, peers, 2, 5)
    us_host = (time.perf_counter() - t0) / 5 * 1e6
    eng.set_verify_mode(0)
    r = {"mode": ["fused", "chain"][mode], "partitions": P, "buckets": B, "peers": R, "peer_bytes": int(off[-1]),
         "device_us_per_call": round(us_dev, 1), "device_partitions_per_s": round(P / us_dev * 1e6),
         "host_api_us_per_call_incl_copies_and_python": round(us_host, 1)}
    print(json.dumps(r), flush=True)
    return r


def bench_decode(eng, n_obj=1, B=1000, cap=1024):
    """Device decode of n_obj EpochTreeObjects of B buckets (mde_decode_epoch_tree_objects_async,
    device-resident inputs and outputs), timed with HIP events."""
    import ctypes as C
    import torch
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7)
    dg = rng.integers(0, 999999, n_obj * B, dtype=np.uint64)
    sz = rng.integers(0, 300, n_obj * B).astype(np.int32)
    objs = eng.encode_objects(B, dg, sz, partition=np.arange(n_obj, dtype=np.int32), lower=5, upper=6)
    off = np.zeros(n_obj + 1, np.int64)
    off[1:] = np.cumsum([len(o) for o in objs])
    blob = torch.from_numpy(np.frombuffer(b"".join(objs), dtype=np.uint8).copy()).to(dev)
    doff = torch.from_numpy(off).to(dev)
    o = [torch.zeros(n_obj, dtype=torch.int32, device=dev), torch.zeros(n_obj, dtype=torch.int64, device=dev),
         torch.zeros(n_obj, dtype=torch.int64, device=dev), torch.zeros(n_obj * cap, dtype=torch.int64, device=dev),
         torch.zeros(n_obj * cap, dtype=torch.int32, device=dev), torch.zeros(n_obj, dtype=torch.uint8, device=dev),
         torch.zeros(n_obj, dtype=torch.int32, device=dev), torch.zeros(n_obj, dtype=torch.int32, device=dev)]
    vp = lambda t: C.c_void_p(t.data_ptr())

    def call():
        rc = eng.lib.mde_decode_epoch_tree_objects_async(eng.ctx, n_obj, vp(blob), vp(doff), cap, *(vp(t) for t in o))
        assert rc == 0, rc

    us = timeit(call, reps=50, warm=5)
    torch.cuda.synchronize()
    assert (o[7].cpu().numpy() == B).all()
    got = o[3].cpu().numpy().view(np.uint64).reshape(n_obj, cap)[:, :B]
    assert (got == dg.reshape(n_obj, B)).all()
    r = {"decode": True, "objects": n_obj, "buckets": B, "cap": cap, "bytes": int(off[-1]), "device_us_per_call": round(us, 2)}
    print(json.dumps(r), flush=True)
    return r


def main():
    import torch
    import mydatastore_amd as mde
    eng = mde.Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    what = sys.argv[1:] or ["tree", "digest"]
    out = {}
    if "tree" in what:
        out["tree"] = bench_tree(eng)
    if "digest" in what:
        out["digest"] = bench_digest(eng)
    if "sweep" in what:
        out["sweep"] = bench_sweep(eng)
    if "verify" in what:
        out["verify"] = [bench_verify(eng, P=p, mode=m) for p in (1, 64, 1024, 8192) for m in (0, 1)]
        out["verify"] += [bench_verify(eng, P=p, B=1000, mode=m) for p in (1, 64) for m in (0, 1)]
    if "decode" in what:
        out["decode"] = [bench_decode(eng, n, B, cap) for n in (1, 1024) for B, cap in ((64, 64), (1000, 1024))]
    for w in what:
        if w.startswith("ab:"):
            out["ab"] = bench_ab(eng, [int(x) for x in w.split(":")[1].split(",")])
        if w.startswith("pieces:"):  # pieces:0,262144,1048576[:c4,c3]
            parts = w.split(":")
            shapes = tuple(parts[2].split(",")) if len(parts) > 2 else ("c4", "c4/8", "c3")
            out["pieces"] = bench_pieces(eng, parts[1].split(","), shapes)
        if w.startswith("stamps:"):  # stamps:ts8k -- probe library only
            out["stamps"] = bench_step_stamps(eng, w.split(":")[1])
        if w.startswith("digestonly:"):  # digestonly:ts8k[:reps] -- the digest kernel alone (PMC runs)
            parts = w.split(":")
            out["digestonly"] = bench_digest_only(eng, parts[1], int(parts[2]) if len(parts) > 2 else 5,
                                                  parts[3] if len(parts) > 3 else "d")
        if w.startswith("fusedonly:"):  # fusedonly:c4bk[:reps] -- fused pipelined builds alone (PMC runs)
            parts = w.split(":")
            out["fusedonly"] = bench_fused_only(eng, parts[1], int(parts[2]) if len(parts) > 2 else 5)
        if w.startswith("digest:"):
            out["digest"] = bench_digest(eng, [int(x) for x in w.split(":")[1].split(",")])
    Path("gpurun_out").mkdir(exist_ok=True)
    Path("gpurun_out/microbench.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
