"""Warm A/B of the production-shape fused step (run once per library, alternating processes):
`warm_ms` of pipelined builds, then K = 40 timed builds in one event bracket, `reps` times in the
process; the last build's roots checked against a standalone build of the same records.
One JSON line: the library, the per-build times, roots_ok.

    MDE_LIBRARY=... [MDE_AB_VARIANT=v] python tools/prod_ab.py [tag] [reps] [warm_ms]
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("MDE_LIBRARY", "shipped")
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    warm_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 40.0
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    if os.environ.get("MDE_AB_VARIANT"):  # an explicit digest variant (e.g. 17: rec8 with 8 KiB steps)
        eng.set_tuning(*map(int, os.environ["MDE_AB_VARIANT"].split(",")))  # variant[,blocks/CU[,oversub]]
        tag += "+v" + os.environ["MDE_AB_VARIANT"]
    # MDE_AB_SHAPE="n_keys,B,value_len,world" (default: the production shape, N = 1)
    n_keys, B, V, world = (int(x) for x in os.environ.get("MDE_AB_SHAPE", "100000000,1000,8,1").split(","))
    if os.environ.get("MDE_AB_SHAPE"):
        tag += "@" + os.environ["MDE_AB_SHAPE"]
    w = make_workload(eng, n_partitions=1024, n_buckets=B, value_len=V, part_mode="mod", n_keys=n_keys,
                      rank=0, world=world)
    sets = [w._outs() for _ in range(2)]
    ref = w.build()["root"].cpu().numpy()

    def builds(k):
        for i in range(k):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])

    t0 = time.perf_counter()
    builds(10)
    eng.build_pipeline_drain_async()
    torch.cuda.synchronize(dev)
    n_warm = max(10, int(warm_ms / ((time.perf_counter() - t0) * 1e3 / 10)))
    us = []
    for _ in range(reps):
        builds(n_warm)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        builds(40)
        b.record(st)
        eng.build_pipeline_drain_async()
        torch.cuda.synchronize(dev)
        us.append(round(a.elapsed_time(b) * 1e3 / 40, 2))
    ok = bool(np.array_equal(sets[1][0]["root"].cpu().numpy(), ref))  # build 39 -> set 1
    dg = []  # the digest kernel alone, warm, 40 launches per bracket
    for _ in range(reps):
        builds(n_warm)
        eng.build_pipeline_drain_async()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(40):
            w.digest_async()
        b.record(st)
        torch.cuda.synchronize(dev)
        dg.append(round(a.elapsed_time(b) * 1e3 / 40, 2))
    print(json.dumps({"lib": tag, "warmup_builds": n_warm, "us_per_build": us, "median_us": float(np.median(us)),
                      "digest_us": dg, "digest_median_us": float(np.median(dg)), "roots_ok": ok}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
