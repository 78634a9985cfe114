"""Where the fused step's waves run (probe build: MDE_WAVE_STAMPS, tools/ab/libmde_stamps.so):
every streaming and tree wave's HW_ID (SIMD, CU, SH, SE) and XCC_ID, for one launch in a warm run
of pipelined builds. Reports how many tree / streaming waves share each SIMD, which SIMD a tree
workgroup's two live waves land on, and the tree waves' exit times by how many tree waves their
SIMD holds. One JSON line per repetition.

    MDE_LIBRARY=tools/ab/libmde_stamps.so python tools/placement_probe.py [n_keys] [B] [value_len] [reps]
"""
import collections
import ctypes
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


def where(v):
    hw, xcc = int(v) & 0xffffffff, int(v) >> 32
    return {"wave": hw & 15, "simd": (hw >> 4) & 3, "cu": (hw >> 8) & 15, "sh": (hw >> 12) & 1,
            "se": (hw >> 13) & 7, "xcc": xcc & 15}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    V = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    if os.environ.get("MDE_AB_VARIANT"):
        eng.set_tuning(int(os.environ["MDE_AB_VARIANT"]), -1)
    w = make_workload(eng, n_partitions=1024, n_buckets=B, value_len=V, part_mode="mod", n_keys=n)
    sets = [w._outs() for _ in range(2)]
    lib = eng.lib
    lib.mde_probe_wave_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    lib.mde_probe_tree_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    lib.mde_probe_hw_where.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    K = 16384
    t0 = time.perf_counter()
    for i in range(10):
        eng.build_pipelined_async(w.rec, sets[i % 2][1])
    eng.build_pipeline_drain_async()
    torch.cuda.synchronize(dev)
    n_warm = max(6, int(40.0 / ((time.perf_counter() - t0) * 1e3 / 10)))
    for rep in range(reps):
        for i in range(n_warm):
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
        wh = np.zeros(K, np.uint64)
        th = np.zeros(K, np.uint64)
        lib.mde_probe_hw_where(wh.ctypes.data, wh.size, 0)
        lib.mde_probe_hw_where(th.ctypes.data, th.size, 1)
        torch.cuda.synchronize(dev)
        st = wb.reshape(-1, 3).astype(np.int64)
        tt = tb.reshape(-1, 2).astype(np.int64)
        s_idx = np.nonzero(st[:, 0] > 0)[0]
        t_idx = np.nonzero((tt[:, 0] > 0) & ((tt[:, 1] - tt[:, 0]) > 100))[0]
        t0s = min(st[s_idx, 0].min(), tt[t_idx, 0].min())
        key = lambda d: (d["xcc"], d["se"], d["sh"], d["cu"], d["simd"])
        tree_per_simd = collections.Counter(key(where(th[i])) for i in t_idx)
        stream_per_simd = collections.Counter(key(where(wh[i])) for i in s_idx)
        simds = set(tree_per_simd) | set(stream_per_simd)
        hist = lambda c: dict(sorted(collections.Counter(c.get(k, 0) for k in simds).items()))
        # the SIMD each live tree wave lands on, by its wave index within the workgroup (tw % 4)
        by_slot = collections.Counter((int(i) % 4, where(th[i])["simd"]) for i in t_idx)
        exit_by_load = collections.defaultdict(list)
        for i in t_idx:
            exit_by_load[tree_per_simd[key(where(th[i]))]].append((tt[i, 1] - t0s) * 10 / 1e3)
        out = {"rep": rep, "shape": [n, B, V], "simds_seen": len(simds), "tree_waves": int(len(t_idx)),
               "stream_waves": int(len(s_idx)),
               "tree_waves_per_simd_hist": {str(k): v for k, v in hist(tree_per_simd).items()},
               "stream_waves_per_simd_hist": {str(k): v for k, v in hist(stream_per_simd).items()},
               "tree_slot_to_simd": {f"{a}->{b}": v for (a, b), v in sorted(by_slot.items())},
               "tree_exit_us_by_trees_on_simd": {str(k): [round(float(np.median(v)), 1), round(float(np.max(v)), 1), len(v)]
                                                 for k, v in sorted(exit_by_load.items())}}
        print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
