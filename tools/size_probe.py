"""Fixed vs per-byte cost of one digest launch at the production value shape (8-byte records,
B = 1,000, 1,024 partitions): the standalone digest kernel timed by HIP events at several arena
sizes; a linear fit gives the per-launch fixed cost and the streaming rate.

    python tools/size_probe.py [n_keys ...]        (MDE_PROBE_B=64 / MDE_PROBE_V=1024: other shapes)
"""
import os
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [25_000_000, 50_000_000, 100_000_000, 200_000_000, 400_000_000]
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    pts = []
    for n in sizes:
        B = int(os.environ.get("MDE_PROBE_B", "1000"))
        V = int(os.environ.get("MDE_PROBE_V", "8"))
        w = make_workload(eng, n_partitions=1024, n_buckets=B, value_len=V, part_mode="mod", n_keys=n // (V // 8),
                          rank=0, world=1)
        w.digest_async()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(20):
            w.digest_async()
        b.record(st)
        torch.cuda.synchronize(dev)
        us = a.elapsed_time(b) * 1e3 / 20
        pts.append((w.value_bytes, us))
        print(json.dumps({"n_keys": n, "bytes": w.value_bytes, "digest_us": round(us, 2),
                          "TBps": round(w.value_bytes / us / 1e6, 3)}), flush=True)
        del w
        torch.cuda.empty_cache()
    x = np.array([p[0] for p in pts], float)
    y = np.array([p[1] for p in pts], float)
    k, c = np.polyfit(x, y, 1)
    print(json.dumps({"fit_fixed_us": round(c, 2), "fit_TBps": round(1 / k / 1e6, 3)}))


if __name__ == "__main__":
    main()
