"""One-partition synchronous builds (the shim's per-call shape) for a rocprofv3 timeline: n 8-byte
LE timestamps at B buckets, K calls of mde_build through the host API; prints the wall time per
call. Run under `rocprofv3 --kernel-trace --memory-copy-trace --stats -- python3 tools/call_trace.py B`.
"""
import json
import sys
import time

from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import mydatastore_amd as mde  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    nodes = bool(int(sys.argv[4])) if len(sys.argv) > 4 else True
    eng = mde.Engine(0)
    rng = np.random.default_rng(1)
    vals = rng.integers(1, 1 << 40, n, dtype=np.uint64).view(np.uint8).copy()
    seg = np.concatenate([[0], np.sort(rng.integers(0, n + 1, B - 1)), [n]]).astype(np.uint64)
    what = sys.argv[5] if len(sys.argv) > 5 else "build"
    if what == "verify":  # the decision step: one agreeing and one differing peer object
        out = eng.build(vals, seg, 1, B, value_stride=8)
        d, z = out["digest"], out["size"]
        d2 = d.copy()
        d2[B // 3] = (d2[B // 3] + 1) % 999999
        peers = eng.encode_objects(B, np.concatenate([d, d2]), np.concatenate([z, z]), lower=3, upper=4)
        call = lambda: eng.verify_epochs(B, d, z, None, [peers], 2, 3, partition=np.array([7], np.int32))
    elif what == "tree":  # the tree alone (tree_kernel from digests): the build minus its digest phase
        dig = eng.build(vals, seg, 1, B, value_stride=8)["digest"]
        call = lambda: eng.tree_from_digests(dig, B, want_nodes=nodes)
    else:
        call = lambda: eng.build(vals, seg, 1, B, value_stride=8, want_nodes=nodes)
    for _ in range(20):
        call()
    t = time.perf_counter()
    for _ in range(K):
        call()
    us = (time.perf_counter() - t) / K * 1e6
    print(json.dumps({"what": what, "B": B, "n": n, "nodes": nodes, "calls": K, "us_per_call": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
