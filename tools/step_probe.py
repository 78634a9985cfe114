"""Per-wave timeline of fused build steps at the production shape (probe build: MDE_WAVE_STAMPS,
`bash tools/build_probe_lib.sh stamps -DMDE_WAVE_STAMPS`, then MDE_LIBRARY=tools/ab/libmde_stamps.so):
for one build_step_kernel launch in a run of pipelined builds, every streaming wave's entry, first
step and exit, and every tree wave's entry and exit (s_memrealtime, 10 ns), relative to the
launch's first wave entry: which role ends the launch, and how far the streaming waves spread.

    MDE_LIBRARY=... python tools/step_probe.py [n_keys] [B] [value_len] [reps]
"""
import ctypes
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    V = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    w = make_workload(eng, n_partitions=1024, n_buckets=B, value_len=V, part_mode="mod", n_keys=n, rank=0, world=1)
    sets = [w._outs() for _ in range(2)]
    lib = eng.lib
    lib.mde_probe_wave_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    lib.mde_probe_tree_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    K = 16384
    for rep in range(reps):
        for i in range(6):  # a run of pipelined builds; the probe reads the launch after the reset
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        torch.cuda.synchronize(dev)
        tb = np.zeros(2 * K, np.uint64)
        lib.mde_probe_tree_stamps(tb.ctypes.data, tb.size, 1)
        eng.build_pipelined_async(w.rec, sets[0][1])
        torch.cuda.synchronize(dev)
        eng.build_pipeline_drain_async()
        wb = np.zeros(3 * K, np.uint64)
        lib.mde_probe_wave_stamps(wb.ctypes.data, wb.size)
        lib.mde_probe_tree_stamps(tb.ctypes.data, tb.size, 0)
        torch.cuda.synchronize(dev)
        st = wb.reshape(-1, 3).astype(np.int64)
        st = st[st[:, 0] > 0]
        tt = tb.reshape(-1, 2).astype(np.int64)
        tt = tt[tt[:, 0] > 0]
        live = tt[(tt[:, 1] - tt[:, 0]) > 100]  # tree waves that built something (> 1 us)
        t0 = min(st[:, 0].min(), tt[:, 0].min())
        us = lambda a: (a - t0) * 10 / 1e3
        e, f, x = us(st[:, 0]), us(st[:, 1]), us(st[:, 2])
        te, tx = us(live[:, 0]), us(live[:, 1])
        q = lambda a, p: round(float(np.percentile(a, p)), 2)
        print(json.dumps({"stream_waves": int(len(st)), "tree_waves": int(len(live)),
                          "span_us": round(float(max(x.max(), tx.max())), 2),
                          "stream_entry_p50": q(e, 50), "stream_entry_max": q(e, 100),
                          "stream_first_p50": q(f, 50), "stream_time_p10": q(x - f, 10), "stream_time_p50": q(x - f, 50),
                          "stream_time_p90": q(x - f, 90), "stream_exit_p10": q(x, 10), "stream_exit_p50": q(x, 50),
                          "stream_exit_p90": q(x, 90), "stream_exit_max": q(x, 100),
                          "tree_entry_p50": q(te, 50), "tree_entry_max": q(te, 100),
                          "tree_time_p50": q(tx - te, 50), "tree_exit_p50": q(tx, 50), "tree_exit_p90": q(tx, 90),
                          "tree_exit_max": q(tx, 100)}), flush=True)


if __name__ == "__main__":
    main()
