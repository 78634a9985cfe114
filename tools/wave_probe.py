"""Per-wave timeline of one standalone digest launch (probe build: MDE_WAVE_STAMPS, e.g.
`bash tools/build_probe_lib.sh stamps -DMDE_WAVE_STAMPS` then MDE_LIBRARY=tools/ab/libmde_stamps.so):
entry, first step and exit of every wave (s_memrealtime, 10 ns), summarised as the dispatch ramp,
the start-up before the first step, the streaming time and the tail.

    MDE_LIBRARY=... python tools/wave_probe.py [n_keys] [B] [value_len]
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
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    w = make_workload(eng, n_partitions=1024, n_buckets=B, value_len=V, part_mode="mod", n_keys=n, rank=0, world=1)
    lib = eng.lib
    lib.mde_probe_wave_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    for rep in range(3):
        for _ in range(5):
            w.digest_async()
        torch.cuda.synchronize(dev)
        buf = np.zeros(3 * 16384, np.uint64)
        lib.mde_probe_wave_stamps(buf.ctypes.data, buf.size)
        buf[:] = 0
        w.digest_async()
        torch.cuda.synchronize(dev)
        lib.mde_probe_wave_stamps(buf.ctypes.data, buf.size)
        st = buf.reshape(-1, 3).astype(np.int64)
        st = st[st[:, 0] > 0]
        t0 = st[:, 0].min()
        e, f, x = (st[:, 0] - t0) * 10 / 1e3, (st[:, 1] - t0) * 10 / 1e3, (st[:, 2] - t0) * 10 / 1e3  # us
        q = lambda a, p: round(float(np.percentile(a, p)), 2)
        print(json.dumps({"waves": int(len(st)), "span_us": q(x, 100), "entry_p50": q(e, 50), "entry_max": q(e, 100),
                          "startup_p50": q(f - e, 50), "startup_p90": q(f - e, 90), "startup_max": q(f - e, 100),
                          "stream_p10": q(x - f, 10), "stream_p50": q(x - f, 50), "stream_p90": q(x - f, 90),
                          "exit_p10": q(x, 10), "exit_p50": q(x, 50), "exit_p90": q(x, 90)}), flush=True)


if __name__ == "__main__":
    main()
