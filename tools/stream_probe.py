#!/usr/bin/env python3
"""How the digest/tree pipelining maps onto HIP streams (probe, not product code).

Times K back-to-back builds of one rank's shard (default: the N=8 shard of C4) under several
stream arrangements and prints ms per build for each:
  serial       digest + tree on one stream
  default+pool digest on the default stream, tree on a pool stream (bench.py's pipeline)
  pool+pool    digest and tree on two created streams
  pool+hiprio  digest on a created stream, tree on a high-priority stream
    python tools/stream_probe.py [world] [steps]
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(world=8, steps=50):
    import torch
    import mydatastore_amd as mde
    from mydatastore_amd.workload import make_workload
    dev = torch.device("cuda", 0)
    e1, e2 = mde.Engine(0), mde.Engine(0)
    w = make_workload(e1, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                      n_keys=10_000_000, rank=0, world=world)
    outs = [w.tree_out, w._outs()[1]]
    engines = [e1, e2]

    def run(main_s, tree_s, timing=0):
        tev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(steps)]
        evd = [torch.cuda.Event() for _ in range(2)]
        evt = [torch.cuda.Event() for _ in range(2)]
        def step(i):
            k = i % 2
            e = engines[k]
            if tree_s is None:
                e.set_stream(main_s.cuda_stream)
                e.digest_async(w.rec)
                e.tree_async(w.rec, outs[k])
                return
            main_s.wait_event(evt[k])
            e.set_stream(main_s.cuda_stream)
            te = timing and i >= 5 and (i - 5) % timing == 0
            if te:
                tev[i - 5][0].record(main_s)
            e.digest_async(w.rec)
            if te:
                tev[i - 5][1].record(main_s)
            evd[k].record(main_s)
            tree_s.wait_event(evd[k])
            e.set_stream(tree_s.cuda_stream)
            e.tree_async(w.rec, outs[k])
            evt[k].record(tree_s)
        for i in range(5):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / steps

    default = torch.cuda.current_stream(dev)
    cfgs = {
        "serial": (default, None),
        "default+pool": (default, torch.cuda.Stream(dev)),
        "pool+pool": (torch.cuda.Stream(dev), torch.cuda.Stream(dev)),
        "pool+hiprio": (torch.cuda.Stream(dev), torch.cuda.Stream(dev, priority=-1)),
        "hiprio+pool": (torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev)),
        "default+pool timing every step": (default, torch.cuda.Stream(dev), 1),
        "default+pool timing every 4th": (default, torch.cuda.Stream(dev), 4),
    }
    for rep in range(2):
        for name, c in cfgs.items():
            ms = run(*c)
            print(json.dumps({"world": world, "arrangement": name, "rep": rep, "ms_per_build": round(ms, 4),
                              "GBps": round(w.value_bytes / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:]))
