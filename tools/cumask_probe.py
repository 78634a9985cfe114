#!/usr/bin/env python3
"""Probe (not product code): pipelined C4 builds with the digest kernel on a CU-masked stream
(224 CUs) and each build's tree kernel on a second stream masked to the other 32 CUs, against the
fused one-launch step and the bare digest kernel, in one process, interleaved.
    python tools/cumask_probe.py [steps]
Needs a probe build whose mde_create reads MDE_PROBE_CUS into the context's CU count (so the
digest grid is planned for 224 CUs); the product library does not carry that hook.
Result (profiles/r02ac_cumask.jsonl): fused 1.48 ms, masked 1.50-1.51 ms per C4 build: rejected.
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def masked_stream(hip, cus, keep):
    words = (cus + 31) // 32
    mask = (C.c_uint32 * words)()
    for c in range(cus):
        if keep(c):
            mask[c // 32] |= 1 << (c % 32)
    st = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(st), C.c_uint32(words), mask)
    assert rc == 0, rc
    return st


def main(steps=20):
    import torch
    import mydatastore_amd as mde
    from mydatastore_amd.workload import make_workload
    dev = torch.device("cuda", 0)
    hip = C.CDLL("libamdhip64.so")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    plain = mde.Engine(0)
    w = make_workload(plain, n_partitions=1024, n_buckets=64, value_len=1024, part_mode="mod",
                      n_keys=10_000_000, rank=0, world=1)
    main_s = torch.cuda.current_stream(dev)
    outs = [w.tree_out, w._outs()[1]]
    layouts = {"last32": lambda c: c >= cus - 32, "every8th": lambda c: c % 8 == 7}
    res = []

    def run(fn, finish):
        for i in range(3):
            fn(i)
        finish()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main_s)
        for i in range(steps):
            fn(i)
        finish()
        b.record(main_s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / steps

    def fused(i):
        plain.set_stream(main_s.cuda_stream)
        plain.build_pipelined_async(w.rec, outs[i % 2])

    def fused_fin():
        plain.set_stream(main_s.cuda_stream)
        plain.build_pipeline_drain_async()

    def digest_only(i):
        plain.set_stream(main_s.cuda_stream)
        plain.digest_async(w.rec)

    setups = {}
    for name, tree_cu in layouts.items():
        os.environ["MDE_PROBE_CUS"] = str(cus - 32)
        e = [mde.Engine(0), mde.Engine(0)]
        os.environ.pop("MDE_PROBE_CUS")
        sa = masked_stream(hip, cus, lambda c, t=tree_cu: not t(c))
        sb = masked_stream(hip, cus, tree_cu)
        ta = torch.cuda.ExternalStream(sa.value, device=dev)
        tb = torch.cuda.ExternalStream(sb.value, device=dev)
        setups[name] = (e, ta, tb)

    def masked(name):
        e, ta, tb = setups[name]
        evd = [torch.cuda.Event() for _ in range(2)]
        evt = [torch.cuda.Event() for _ in range(2)]
        start = torch.cuda.Event()

        def fn(i):
            k = i % 2
            if i == 0:
                start.record(main_s)
                ta.wait_event(start)
            ta.wait_event(evt[k])
            e[k].set_stream(ta.cuda_stream)
            e[k].digest_async(w.rec)
            evd[k].record(ta)
            tb.wait_event(evd[k])
            e[k].set_stream(tb.cuda_stream)
            e[k].tree_async(w.rec, outs[k])
            evt[k].record(tb)

        def fin():
            main_s.wait_event(evt[0])
            main_s.wait_event(evt[1])
            main_s.wait_stream(ta)
        return fn, fin

    ref = None
    for rep in range(3):
        for mode in ("digest_only", "fused") + tuple("masked_" + n for n in layouts):
            if mode == "digest_only":
                ms = run(digest_only, lambda: None)
            elif mode == "fused":
                ms = run(fused, fused_fin)
            else:
                fn, fin = masked(mode[len("masked_"):])
                ms = run(fn, fin)
            r = {"mode": mode, "rep": rep, "ms_per_build": round(ms, 4), "GBps": round(w.value_bytes / ms / 1e6, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
    # parity: the masked pipeline's roots equal a plain build's
    o = w.build()
    fn, fin = masked("last32")
    for i in range(2):
        fn(i)
    fin()
    torch.cuda.synchronize()
    ok = bool(torch.equal(w.out["root"], o["root"]))  # build 0 wrote output set 0 (w.out)
    print(json.dumps({"masked_roots_equal_plain_build": ok}), flush=True)


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:2]))
