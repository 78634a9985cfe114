"""Why the production-shape fused step reads 150-172 us per build in bench.py's production_shape
probe but ~190 us in the `--config prod` line of the same process (gpurun_out/r05n).

Two 800 MB PROD_SHAPE workloads (allocated one after the other) are timed alternately, each with
  bracket_K  the bench line's method: synchronize, one event pair around K pipelined builds
             (the drain outside), ms / K;
  diff       production_shape's method: a run of 2n minus a run of n, each right after a warm run
             (no idle gap before the timed launches).
K in {10, 20, 40} separates a per-run fixed cost (start from an idle GPU) from the per-build time.
One JSON line per measurement.

    python tools/prod_var.py [reps]
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    ws = []
    for _ in range(2):
        w = make_workload(eng, n_partitions=1024, n_buckets=1000, value_len=8, part_mode="mod", n_keys=100_000_000)
        ws.append((w, [w._outs() for _ in range(2)]))
    torch.cuda.synchronize(dev)

    def run(w, sets, n):
        for i in range(n):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        eng.build_pipeline_drain_async()

    def bracket(w, sets, k, idle_ms=0.0):
        run(w, sets, 3)
        torch.cuda.synchronize(dev)
        if idle_ms:
            time.sleep(idle_ms / 1e3)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for i in range(k):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        b.record(st)
        eng.build_pipeline_drain_async()
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) * 1e3 / k

    def timed(fn):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) * 1e3

    for rep in range(reps):
        for wi, (w, sets) in enumerate(ws):
            out = {"rep": rep, "workload": wi, "values_ptr_mod_2M": w.values.data_ptr() % (2 << 20)}
            for k in (10, 20, 40):
                out[f"bracket_{k}_us"] = round(bracket(w, sets, k), 2)
            out["bracket_20_after_50ms_idle_us"] = round(bracket(w, sets, 20, 50.0), 2)
            t1 = timed(lambda: run(w, sets, 10))
            t2 = timed(lambda: run(w, sets, 20))
            out["diff_us"] = round((t2 - t1) / 10, 2)
            out["run10_us"] = round(t1 / 10, 2)
            print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
