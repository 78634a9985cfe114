"""bench.py's production_shape measurement alone, 3 times in a fresh process (after an optional
C4-sized warm-up of the device), to separate the measurement from the bench's preceding C4 run."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import mydatastore_amd as mde  # noqa: E402


def main():
    warm = len(sys.argv) > 1 and sys.argv[1] == "warm"
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    if warm:  # ~1 s of C4-sized streaming first
        from mydatastore_amd.workload import make_workload
        w = make_workload(eng, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                          n_keys=10_000_000, rank=0, world=1)
        for _ in range(600):
            w.digest_async()
        torch.cuda.synchronize(dev)
        del w
        torch.cuda.empty_cache()
    for _ in range(3):
        r = bench.production_shape(torch, eng, dev, 16)
        print(json.dumps({"warm": warm, "fused_us": r["fused_us_per_build"], "digest_us": r["digest_kernel_us"],
                          "ok": r["equals_c_oracle_on_sample"]}), flush=True)


if __name__ == "__main__":
    main()
