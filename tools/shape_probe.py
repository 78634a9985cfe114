"""Where a fused build's time goes for one shape, warm (after >= warm_ms of builds): K fused
pipelined builds, K standalone digests (the same digest form, no trees) and K standalone tree
passes (tree_async over the digests already in the engine's slot), each in one event bracket;
`reps` alternations. One JSON line per repetition.

    python tools/shape_probe.py [n_keys] [P] [value_len] [B] [reps] [warm_ms]
    (defaults: C4 at B = 1,000 -- the reference's default PartitionBuckets over C4's data)
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:5]] + [0] * (4 - len(sys.argv[1:5]))
    n = a[0] or 10_000_000
    P = a[1] or 1024
    V = a[2] or 1024
    B = a[3] or 1000
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    warm_ms = float(sys.argv[6]) if len(sys.argv) > 6 else 40.0
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)
    w = make_workload(eng, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n)
    sets = [w._outs() for _ in range(2)]
    K = 20

    def fused(k):
        for i in range(k):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])

    def bracket(fn):
        x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        x.record(st)
        fn()
        y.record(st)
        torch.cuda.synchronize(dev)
        return x.elapsed_time(y) * 1e3 / K

    t0 = time.perf_counter()
    fused(3)
    eng.build_pipeline_drain_async()
    torch.cuda.synchronize(dev)
    n_warm = max(3, int(warm_ms / ((time.perf_counter() - t0) * 1e3 / 3)))
    for rep in range(reps):
        fused(n_warm)
        f_us = bracket(lambda: fused(K))
        eng.build_pipeline_drain_async()
        d_us = bracket(lambda: [w.digest_async() for _ in range(K)])
        t_us = bracket(lambda: [w.tree_async(sets[0][1]) for _ in range(K)])
        print(json.dumps({"shape": [n, P, V, B], "rep": rep, "warmup_builds": n_warm, "fused_us": round(f_us, 2),
                          "digest_us": round(d_us, 2), "tree_us": round(t_us, 2),
                          "fused_frac": round(w.value_bytes / f_us / 1e3 / 8000.0, 4),
                          "digest_frac": round(w.value_bytes / d_us / 1e3 / 8000.0, 4)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
