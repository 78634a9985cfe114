"""Full-size equality of digest variants on the production shape (100 M 8-byte values, 1,024
partitions, B = 1,000) and its N = 8 shard: every listed variant's standalone and fused builds
equal the default build in digests, sizes, items, roots and nodes (the default's parity with the C
oracle is tests/test_configs.py PROD). One JSON line per (world, variant).

    python tools/rec8_variant_check.py 19 20
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    variants = [int(v) for v in sys.argv[1:]] or [19, 20]
    eng = mde.Engine(0)
    eng.set_stream(torch.cuda.current_stream(torch.device("cuda:0")).cuda_stream)
    for world in (1, 8):
        w = make_workload(eng, n_partitions=1024, n_buckets=1000, value_len=8, part_mode="mod",
                          n_keys=100_000_000, rank=0, world=world)
        ref = w.build()
        for v in variants:
            eng.set_tuning(v, -1)
            ok = {}
            for fused in (False, True):
                if fused:
                    o, to = w._outs()
                    for _ in range(3):
                        eng.build_pipelined_async(w.rec, to)
                    eng.build_pipeline_drain_async()
                    eng.synchronize()
                else:
                    o = w.build()
                ok["fused" if fused else "standalone"] = all(torch.equal(o[k], ref[k])
                                                             for k in ("digest", "size", "items", "root", "nodes"))
            eng.set_tuning(-1, -1)
            print(json.dumps({"world": world, "variant": v, **ok}), flush=True)
            if not all(ok.values()):
                sys.exit(1)
        del w
    eng.close()


if __name__ == "__main__":
    main()
