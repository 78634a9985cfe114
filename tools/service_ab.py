"""The resident build service's cost to bulk builds on the same device.

A node runs VerifyEpoch's one-partition calls through the resident service (INTEGRATION.md
section 3) while it also rebuilds whole epochs in bulk (mde_build_pipelined_async). The service's
launch keeps one workgroup per request slot resident for its lifetime (100 ms after each call), so
the bulk builds share the CUs with it. This times runs of fused pipelined builds (HIP events on
the engine's stream) in three states, alternating, `reps` times:
  none     no service on the device;
  idle     a live service whose launch is resident and polling (one call just before the run);
  serving  the same service serving `callers` threads of one-partition builds (1,000 8-byte
           timestamps, B = 1,000: the reference's production call) throughout the run.
One JSON line per state and repetition: ms per bulk build, and for `serving` the calls served.

    python tools/service_ab.py [c4|prod] [reps] [callers] [builds]
"""
import json
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402

SHAPES = {"c4": (10_000_000, 1024, 1024, 64), "prod": (100_000_000, 1024, 8, 1000)}


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c4"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    callers = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    builds = int(sys.argv[4]) if len(sys.argv) > 4 else (20 if shape == "c4" else 100)
    n, P, V, B = SHAPES[shape]
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    w = make_workload(eng, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n)
    sets = [w._outs() for _ in range(2)]
    ref = w.build()["root"].cpu().numpy()

    def run(k):
        for i in range(k):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        eng.build_pipeline_drain_async()

    def timed():
        run(2)
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        run(builds)
        b.record(st)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) / builds

    # one-partition calls: 1,000 LE64 timestamps over B = 1,000 buckets
    rng = np.random.default_rng(7)
    one_vals = (1_700_000_000 + np.cumsum(rng.integers(1, 8, 1000))).astype(np.uint64).view(np.uint8).copy()
    one_seg = (np.arange(1001, dtype=np.uint64) * 1000 // 1000).astype(np.uint64)
    sv = mde.Server(0)
    served = [0]
    stop = threading.Event()

    def caller():
        while not stop.is_set():
            sv.build(one_vals, one_seg, 1, 1000, value_stride=8, want_nodes=False)
            served[0] += 1

    for rep in range(reps):
        for state in ("none", "idle", "serving"):
            th = []
            if state == "idle":
                sv.build(one_vals, one_seg, 1, 1000, value_stride=8, want_nodes=False)  # launch resident
            elif state == "serving":
                stop.clear()
                served[0] = 0
                th = [threading.Thread(target=caller) for _ in range(callers)]
                for t in th:
                    t.start()
                time.sleep(0.02)
            if state == "none":
                time.sleep(0.25)  # the service's launch has ended its 100 ms lifetime
            c0 = served[0]
            ms = timed()
            c1 = served[0]
            stop.set()
            for t in th:
                t.join()
            ok = bool(np.array_equal(sets[(builds - 1) % 2][0]["root"].cpu().numpy(), ref))
            line = {"shape": shape, "rep": rep, "state": state, "ms_per_build": round(ms, 5), "roots_ok": ok,
                    "launches": sv.stats()["launches"]}
            if state == "serving":
                line["calls_during_run"] = c1 - c0
                line["callers"] = callers
            print(json.dumps(line), flush=True)
    sv.close()
    eng.close()


if __name__ == "__main__":
    main()
