"""How much untimed load the GPU needs after an idle spell before a timed run of builds reads its
steady-state rate (gpurun_out/r05o: the production-shape step reads ~170 us per build right after
other GPU work, ~190 us after 50 ms idle -- the clock ramps down when the device idles).

For C4 and the production shape: idle for `idle_s` (as bench.py's host-side parity checks leave the
device before its warmup), then W untimed pipelined builds, synchronize, then K = 20 timed builds
(one event pair, bench.py's bracket). W in {0, 3, 10, 30, 100}; plus a control with no idle.
One JSON line per (shape, rep, W).

    python tools/clock_ramp.py [reps] [idle_s]
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402

SHAPES = {"c4": (10_000_000, 1024, 1024, 64), "prod": (100_000_000, 1024, 8, 1000)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    idle_s = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    for shape in ("prod", "c4"):
        n, P, V, B = SHAPES[shape]
        w = make_workload(eng, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n)
        sets = [w._outs() for _ in range(2)]

        def builds(k):
            for i in range(k):
                eng.build_pipelined_async(w.rec, sets[i % 2][1])

        def measure(warm, idle):
            if idle:
                time.sleep(idle)
            builds(warm)
            eng.build_pipeline_drain_async()
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            builds(20)
            b.record(st)
            eng.build_pipeline_drain_async()
            torch.cuda.synchronize(dev)
            return a.elapsed_time(b) * 1e3 / 20

        measure(3, 0)
        for rep in range(reps):
            for warm in (0, 3, 10, 30, 100):
                us = measure(warm, idle_s)
                print(json.dumps({"shape": shape, "rep": rep, "idle_s": idle_s, "warmup_builds": warm,
                                  "us_per_build": round(us, 2)}), flush=True)
            us = measure(3, 0)
            print(json.dumps({"shape": shape, "rep": rep, "idle_s": 0, "warmup_builds": 3,
                              "us_per_build": round(us, 2)}), flush=True)
        del w, sets
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
