#!/usr/bin/env python3
"""A/B of build pipelining modes in ONE process (probe, not product code): ms per build for
digest-only, fused (mde_build_pipelined_async) and two-stream pipelining, interleaved 3 times.
    python tools/pipe_probe.py [world] [steps] [layout a|b]
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(world=1, steps=20, layout="a"):
    import torch
    import mydatastore_amd as mde
    from mydatastore_amd.workload import make_workload
    dev = torch.device("cuda", 0)
    e1, e2 = mde.Engine(0), mde.Engine(0)
    w = make_workload(e1, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                      n_keys=10_000_000, rank=0, world=world, layout=layout)
    main_s = torch.cuda.current_stream(dev)
    tree_s = torch.cuda.Stream(dev)
    outs = [w.tree_out, w._outs()[1]]
    evd = [torch.cuda.Event() for _ in range(2)]
    evt = [torch.cuda.Event() for _ in range(2)]

    def timed(fn, finish=None):
        for i in range(3):
            fn(i)
        if finish:
            finish()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main_s)
        for i in range(steps):
            fn(i)
        if finish:
            finish()
        b.record(main_s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / steps

    def digest_only(i):
        e1.set_stream(main_s.cuda_stream)
        e1.digest_async(w.rec)

    def fused(i):
        e1.set_stream(main_s.cuda_stream)
        e1.build_pipelined_async(w.rec, outs[i % 2])

    def streams(i):
        k = i % 2
        e = (e1, e2)[k]
        main_s.wait_event(evt[k])
        e.set_stream(main_s.cuda_stream)
        e.digest_async(w.rec)
        evd[k].record(main_s)
        tree_s.wait_event(evd[k])
        e.set_stream(tree_s.cuda_stream)
        e.tree_async(w.rec, outs[k])
        evt[k].record(tree_s)

    def streams_join():
        main_s.wait_event(evt[0])
        main_s.wait_event(evt[1])

    side = torch.cuda.Stream(dev)
    evb = [torch.cuda.Event() for _ in range(2)]
    evg = [torch.cuda.Event() for _ in range(2)]
    slab = torch.zeros(32 * 1024, dtype=torch.uint8, device=dev)
    gat = torch.zeros(8 * 32 * 1024, dtype=torch.uint8, device=dev)

    def fused_side(i, bucket=1):
        # bench.py's N>1 event pattern (one side-stream hand-off per `bucket` builds), with a
        # device copy standing in for the RCCL gather
        if i >= 1 and (i - 1) % bucket == 0:
            main_s.wait_event(evg[((i - 1) // bucket) % 2])
        e1.set_stream(main_s.cuda_stream)
        e1.build_pipelined_async(w.rec, outs[i % 2])
        if i >= 1 and i % bucket == 0:
            k = ((i - 1) // bucket) % 2
            evb[k].record(main_s)
            side.wait_event(evb[k])
            with torch.cuda.stream(side):
                gat.view(8, -1).copy_(slab.expand(8, -1))
                evg[k].record(side)

    def serial(i):
        e1.set_stream(main_s.cuda_stream)
        e1.digest_async(w.rec)
        e1.tree_async(w.rec, outs[i % 2])

    for rep in range(3):
        for name, fn, fin in (("digest_only", digest_only, None),
                              ("fused", fused, lambda: (e1.set_stream(main_s.cuda_stream), e1.build_pipeline_drain_async())),
                              ("fused+side", fused_side, lambda: (e1.set_stream(main_s.cuda_stream), e1.build_pipeline_drain_async(), main_s.wait_stream(side))),
                              ("fused+side/4", lambda i: fused_side(i, 4), lambda: (e1.set_stream(main_s.cuda_stream), e1.build_pipeline_drain_async(), main_s.wait_stream(side))),
                              ("streams", streams, streams_join), ("serial", serial, None)):
            ms = timed(fn, fin)
            print(json.dumps({"world": world, "layout": layout, "mode": name, "rep": rep, "ms_per_build": round(ms, 4),
                              "GBps": round(w.value_bytes / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*(int(x) for x in a[:2]), *a[2:3])
