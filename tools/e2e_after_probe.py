"""What the end-to-end leg leaves behind (r06s: bench's production-shape digest alone reads 155-159
us after `end_to_end`, 140 without it). One process, the production workload's standalone
digest (40 launches per bracket, warm) and fused step measured: fresh; the same workload after
bench.end_to_end (C4 streamed from pinned host memory); a workload allocated after it, while
torch's device cache holds end_to_end's 10 GB buffer; one allocated after releasing the cache; one
carved from a freed 10 GB torch block without end_to_end. (r06t: pinned host buffers, device
alloc/free and end_to_end itself leave the already-allocated workload's digest at 140-143 us.)

    python tools/e2e_after_probe.py
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import mydatastore_amd as mde  # noqa: E402
from mydatastore_amd.workload import make_workload  # noqa: E402


def main():
    eng = mde.Engine(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    eng.set_stream(st.cuda_stream)

    def prod():
        w = make_workload(eng, n_partitions=1024, n_buckets=1000, value_len=8, part_mode="mod",
                          n_keys=100_000_000, rank=0, world=1)
        return w, [w._outs() for _ in range(2)]

    w, sets = prod()

    def fused(n):
        for i in range(n):
            eng.build_pipelined_async(w.rec, sets[i % 2][1])
        eng.build_pipeline_drain_async()

    def digests(n):
        for _ in range(n):
            w.digest_async()

    def bracket(fn, n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn(n)
        b.record(st)
        torch.cuda.synchronize(dev)
        return round(a.elapsed_time(b) * 1e3 / n, 2)

    def measure(case):
        fused(150)
        d = [bracket(digests, 40) for _ in range(3)]
        fused(50)
        f = bracket(fused, 40)
        print(json.dumps({"case": case, "digest_us": d, "fused_us_incl_drain": f}), flush=True)

    def host_empty():
        torch.cuda.synchronize(dev)
        if hasattr(torch._C, "_host_emptyCache"):
            torch._C._host_emptyCache()

    ps = lambda tag: print(json.dumps({"case": tag, "production_shape": {
        k: v for k, v in bench.production_shape(torch, eng, dev, 16).items()
        if k in ("fused_us_per_build", "digest_kernel_us", "equals_c_oracle_on_sample")}}), flush=True)
    ps("bench.production_shape, fresh")
    c4 = make_workload(eng, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                       n_keys=10_000_000, rank=0, world=1)
    g = mde.Group([0])
    print(json.dumps({"gather_kind": g.gather_kind}), flush=True)
    c4_sets = [c4._outs()[0] for _ in range(2)]
    send = torch.zeros(8 * 1024 * 32, dtype=torch.uint8, device=dev)
    recv = torch.zeros_like(send)

    def tree_out(o, root):
        return mde.TreeOut(o["digest"].data_ptr(), o["size"].data_ptr(), o["items"].data_ptr(), root,
                           o["nodes"].data_ptr())

    def group_run(n):
        for L in range(n):
            g.build_async([c4.rec], [tree_out(c4_sets[L % 2], send.data_ptr() + (L % 8) * 1024 * 32)], pipelined=True)
            if L % 8 == 7:
                g.gather_wait_async(g.gather_overlapped_async([send], [recv], send.numel()))
        g.drain_async()
        g.synchronize()

    group_run(40)
    ps("after group builds + RCCL gathers on the C4 shard")
    e = bench.end_to_end(torch, eng, c4, 64, reps=1)
    print(json.dumps({"end_to_end": e}), flush=True)
    ps("after group + end_to_end")
    g.close()
    ps("after group + end_to_end, group closed")
    eng.close()


if __name__ == "__main__":
    main()
