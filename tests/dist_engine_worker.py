"""One rank of the two-process engine test (tests/test_group.py): launched by torch.distributed.run
with gloo, every rank on cuda:0 (the one GPU of the box), fresh processes started before any GPU
call. Each rank builds ITS shard (partition p on rank p % world) with the engine, the roots are
all-gathered (gloo, staged through the host), and rank 0 compares the assembled roots, and a
sample of digests, with ONE engine build of the whole workload in the same process. Prints one
JSON line on rank 0."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import mydatastore_amd as mde
    from mydatastore_amd.dist import RootGather
    from mydatastore_amd.workload import make_workload
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    P, B, V, n = 96, 64, 64, 200_000
    eng = mde.Engine(0)
    w = make_workload(eng, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n, rank=rank, world=world)
    out = w.build()
    g = RootGather(P, world, torch.device("cpu"))
    g.gather(out["root"].cpu(), 0)
    allr = g.assemble(0)
    ok = True
    if rank == 0:
        whole = make_workload(eng, n_partitions=P, n_buckets=B, value_len=V, part_mode="mod", n_keys=n)
        ref = whole.build()
        want = ref["root"].cpu().numpy().reshape(P, 32)
        ok = bool(np.array_equal(allr, want))
        mine = ref["digest"].cpu().numpy().reshape(P, B)[w.partition_ids]
        ok_dig = bool(np.array_equal(out["digest"].cpu().numpy().reshape(-1, B), mine))
        print(json.dumps({"world": world, "gathered_roots_equal_single_process": ok,
                          "rank0_digests_equal_single_process": ok_dig,
                          "engine": str(mde.load_library()._name)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
