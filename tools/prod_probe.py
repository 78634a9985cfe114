"""Production-shape probe: the 8-byte-timestamp, B = 1,000 workload (bench.py PROD_SHAPE) built
under several digest tunings -- variant, resident workgroups per CU -- with the standalone digest
kernel and the fused pipelined step timed by HIP events, every tuning's outputs compared with the
default's. One JSON line per tuning.

    python tools/prod_probe.py [variant,blocks_per_cu[,oversub] ...]     (default: a small sweep)
    MDE_LIBRARY=<-DMDE_STEP_STAMPS build> python tools/prod_probe.py stamps
                 (per fused step: when the tree waves and the stream waves finished)
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def stamps(eng, w, sets, reps=8):
    import ctypes as C
    fn = eng.lib.mde_probe_step_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    buf = (C.c_ulonglong * 4)()
    for i in range(reps + 2):
        torch.cuda.synchronize()
        fn(buf, 1)
        eng.build_pipelined_async(w.rec, sets[i % 2][1])
        torch.cuda.synchronize()
        fn(buf, 0)
        t = list(buf)
        if i >= 2:
            z = min(t[0], t[2])
            print(json.dumps({"tree_start_us": round((t[0] - z) / 100, 2), "tree_end_us": round((t[1] - z) / 100, 2),
                              "stream_start_us": round((t[2] - z) / 100, 2), "stream_end_us": round((t[3] - z) / 100, 2)}),
                  flush=True)
    eng.build_pipeline_drain_async()
    torch.cuda.synchronize()


def main():
    if sys.argv[1:] == ["stamps"]:
        eng = mde.Engine(0)
        n_keys, P, V, B, mode, _ = bench.PROD_SHAPE
        w = make_workload(eng, n_partitions=P, n_buckets=B, value_len=V, part_mode=mode, n_keys=n_keys, rank=0, world=1)
        stamps(eng, w, [w._outs() for _ in range(2)])
        return
    tunings = [tuple(map(int, a.split(","))) for a in sys.argv[1:]] or [(-1, -1), (15, 3), (15, 4), (16, 3), (16, 4)]
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    n_keys, P, V, B, mode, _ = bench.PROD_SHAPE
    w = make_workload(eng, n_partitions=P, n_buckets=B, value_len=V, part_mode=mode, n_keys=n_keys, rank=0, world=1)
    sets = [w._outs() for _ in range(2)]
    ref = None

    def timed(fn, reps):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) * 1e3 / reps

    def run(n):
        for i in range(n):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        eng.build_pipeline_drain_async()

    for t in tunings:
        v, bpc, osub = (t + (-1,))[:3]
        eng.set_tuning(v, bpc, osub)
        digest_us = timed(w.digest_async, 20)
        t1 = timed(lambda: run(10), 1)
        t2 = timed(lambda: run(20), 1)
        fused_us = (t2 - t1) / 10
        run(1)
        torch.cuda.synchronize(dev)
        got = {k: sets[0][0][k].clone() for k in ("digest", "size", "items", "root")}
        if ref is None:
            ref = got
        same = all(torch.equal(got[k], ref[k]) for k in got)
        print(json.dumps({"variant": v, "blocks_per_cu": bpc, "oversub": osub, "digest_us": round(digest_us, 2),
                          "digest_frac": round(w.value_bytes / digest_us / 1e3 / 8000, 4),
                          "fused_us": round(fused_us, 2), "fused_frac": round(w.value_bytes / fused_us / 1e3 / 8000, 4),
                          "equals_default": same}), flush=True)
    eng.set_tuning(-1, -1)


if __name__ == "__main__":
    main()
