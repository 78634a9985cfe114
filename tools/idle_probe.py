"""Is the production-shape digest alone slow after the GPU idles (bench.py runs it after the
CPU baseline's ~10 s with an idle GPU)? The standalone digest kernel (40 launches per bracket)
timed: busy; after an idle spell with bench's fused warm-up (>= 25 ms); after the same idle with
a digest-only warm-up; after the idle with a 250 ms fused warm-up. One JSON line per case.

    python tools/idle_probe.py [idle_s]
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    idle_s = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    w = make_workload(eng, n_partitions=1024, n_buckets=1000, value_len=8, part_mode="mod", n_keys=100_000_000,
                      rank=0, world=1)
    sets = [w._outs() for _ in range(2)]

    def fused(n):
        for i in range(n):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        eng.build_pipeline_drain_async()

    def digests(n):
        for _ in range(n):
            w.digest_async()

    def bracket(fn, n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn(n)
        b.record(st)
        torch.cuda.synchronize(dev)
        return round(a.elapsed_time(b) * 1e3 / n, 2)

    fused(200)
    torch.cuda.synchronize(dev)
    cases = [("busy", None, 0), ("idle+fused25ms", fused, 25), ("idle+digest25ms", digests, 25),
             ("idle+fused250ms", fused, 250), ("idle+none", None, 0)]
    for rep in range(2):
        for name, warm, ms in cases:
            if name != "busy":
                torch.cuda.synchronize(dev)
                time.sleep(idle_s)
            if warm is not None:
                per = 0.17 if warm is fused else 0.14  # ms per launch, roughly
                warm(max(1, int(ms / per)))
            d = bracket(digests, 40)
            f = bracket(fused, 40)
            print(json.dumps({"rep": rep, "case": name, "idle_s": idle_s if name != "busy" else 0,
                              "digest_us": d, "fused_us_after": f}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
