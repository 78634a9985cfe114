"""What the wide trees' top levels cost the production-shape fused step: steady-state fused builds
(bench.py production_shape's method: a run of 2n pipelined builds minus a run of n, HIP events) of
100 M 8-byte values at B = 1,000 with the library in MDE_LIBRARY. Built with
-DMDE_PROBE_STEP_TOP_NODES=64 (tools/build_probe_lib.sh), every fused tree stops at its first level of
at most 64 nodes (wrong roots: timing only), which bounds what packing those levels could gain.

    MDE_LIBRARY=... python tools/top_probe.py [label] [reps]
"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("MDE_LIBRARY", "default")
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n_keys, P, V, B, mode, _ = bench.PROD_SHAPE
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    w = make_workload(eng, n_partitions=P, n_buckets=B, value_len=V, part_mode=mode, n_keys=n_keys)
    sets = [w._outs() for _ in range(2)]

    def run(n):
        for i in range(n):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        eng.build_pipeline_drain_async()

    def timed(fn):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) * 1e3

    for r in range(reps):
        k = 20
        us = (timed(lambda: run(2 * k)) - timed(lambda: run(k))) / k
        print(json.dumps({"lib": label, "rep": r, "fused_us_per_build": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
