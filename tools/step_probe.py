"""Per-wave timeline of fused build steps at the production shape (probe build: MDE_WAVE_STAMPS,
`bash tools/build_probe_lib.sh stamps -DMDE_WAVE_STAMPS`, then MDE_LIBRARY=tools/ab/libmde_stamps.so):
for one build_step_kernel launch in a run of pipelined builds, every streaming wave's entry, first
step and exit, and every tree wave's entry and exit (s_memrealtime, 10 ns), relative to the
launch's first wave entry: which role ends the launch, and how far the streaming waves spread.
Each wave's shader clock over its life too (s_memtime cycles / s_memrealtime time). `warm_ms`: the
probed launch follows that much device time of pipelined builds (0: a short run after an idle
spell of `idle_s`), to read the clock the step sustains against the one it starts at.

    MDE_LIBRARY=... python tools/step_probe.py [n_keys] [B] [value_len] [reps] [warm_ms] [idle_s]
"""
import os
import time
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
    warm_ms = float(sys.argv[5]) if len(sys.argv) > 5 else 0.0
    idle_s = float(sys.argv[6]) if len(sys.argv) > 6 else 0.0
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    if os.environ.get("MDE_AB_VARIANT"):
        eng.set_tuning(int(os.environ["MDE_AB_VARIANT"]), -1)
    w = make_workload(eng, n_partitions=1024, n_buckets=B, value_len=V, part_mode="mod", n_keys=n, rank=0, world=1)
    sets = [w._outs() for _ in range(2)]
    lib = eng.lib
    lib.mde_probe_wave_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    lib.mde_probe_tree_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    lib.mde_probe_clock_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    K = 16384
    for i in range(6):
        eng.build_pipelined_async(w.rec, sets[i % 2][1])
    eng.build_pipeline_drain_async()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(10):
        eng.build_pipelined_async(w.rec, sets[i % 2][1])
    eng.build_pipeline_drain_async()
    torch.cuda.synchronize(dev)
    n_warm = max(6, int(warm_ms / ((time.perf_counter() - t0) * 1e3 / 10))) if warm_ms else 6
    for rep in range(reps):
        if idle_s:
            time.sleep(idle_s)
        for i in range(n_warm):  # a run of pipelined builds; the probe reads the launch after the reset
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
        wc = np.zeros(3 * K, np.uint64)
        tc = np.zeros(2 * K, np.uint64)
        lib.mde_probe_clock_stamps(wc.ctypes.data, wc.size, 0)
        lib.mde_probe_clock_stamps(tc.ctypes.data, tc.size, 1)
        torch.cuda.synchronize(dev)
        # per-wave shader clock (MHz) over entry -> exit: cycles / (10 ns ticks) x 100
        sm = wb.reshape(-1, 3)[:, 0] > 0
        wcl = wc.reshape(-1, 3).astype(np.int64)[sm]
        wrt = wb.reshape(-1, 3).astype(np.int64)[sm]
        s_mhz = (wcl[:, 2] - wcl[:, 0]) / np.maximum(wrt[:, 2] - wrt[:, 0], 1) * 100.0
        tm = tb.reshape(-1, 2)[:, 0] > 0
        tcl = tc.reshape(-1, 2).astype(np.int64)[tm]
        trt = tb.reshape(-1, 2).astype(np.int64)[tm]
        tlive = (trt[:, 1] - trt[:, 0]) > 100
        t_mhz = (tcl[tlive, 1] - tcl[tlive, 0]) / (trt[tlive, 1] - trt[tlive, 0]) * 100.0
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
        print(json.dumps({"warmup_builds": n_warm, "idle_s": idle_s,
                          "stream_clock_mhz_p10": q(s_mhz, 10), "stream_clock_mhz_p50": q(s_mhz, 50),
                          "stream_clock_mhz_p90": q(s_mhz, 90), "tree_clock_mhz_p10": q(t_mhz, 10),
                          "tree_clock_mhz_p50": q(t_mhz, 50), "tree_clock_mhz_p90": q(t_mhz, 90),
                          "stream_waves": int(len(st)), "tree_waves": int(len(live)),
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
