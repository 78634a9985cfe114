#!/usr/bin/env python3
"""Device occupancy of a rocprofv3 --kernel-trace [--memory-copy-trace] run: the fraction of the
traced span with 0, 1, 2, ... kernels (and copies) in flight, and the median kernel / copy times --
where a batch of one-partition calls spends its time (tests/cpp/batch_bench.c).

    python tools/trace_busy.py <dir with *_kernel_trace.csv> [kernel-name substring]
"""
import csv
import glob
import json
import statistics
import sys


def intervals(pattern, name_key, sub):
    fs = sorted(glob.glob(pattern, recursive=True))
    if not fs:
        return []
    rows = list(csv.DictReader(open(fs[0], newline="")))
    return [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
            if not sub or sub in r.get(name_key, "")]


def occupancy(iv):
    if not iv:
        return {}, 0
    ev = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv])
    t0, t1 = ev[0][0], ev[-1][0]
    hist, cur, last = {}, 0, t0
    for t, d in ev:
        hist[cur] = hist.get(cur, 0) + (t - last)
        cur += d
        last = t
    span = max(t1 - t0, 1)
    return {k: round(v / span, 3) for k, v in sorted(hist.items())}, span


def main(d, sub=""):
    ks = intervals(f"{d}/**/*kernel_trace.csv", "Kernel_Name", sub)
    cs = intervals(f"{d}/**/*memory_copy_trace.csv", "Direction", "")
    occ, span = occupancy(ks)
    both, _ = occupancy(ks + cs)
    out = {"kernels": len(ks), "span_ms": round(span / 1e6, 3),
           "kernel_median_us": round(statistics.median([(e - s) / 1e3 for s, e in ks]), 2) if ks else None,
           "copies": len(cs),
           "copy_median_us": round(statistics.median([(e - s) / 1e3 for s, e in cs]), 2) if cs else None,
           "fraction_of_span_with_k_kernels": occ, "fraction_with_k_kernels_or_copies": both}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
