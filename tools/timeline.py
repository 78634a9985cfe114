#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 --kernel-trace run: per-kernel durations and the gaps between
consecutive launches of the dominant kernel (where a bench step loses time outside the kernel).

    python tools/timeline.py <dir with *_kernel_trace.csv> [last_n]
"""
import csv
import glob
import statistics
import sys


def short(name):
    for k in ("build_step_kernel", "bucket_digest_kernel", "tagged_digest_kernel", "tree_kernel", "diff_kernel",
              "synth", "tag_keys_kernel", "verify_kernel", "encode_kernel", "decode_kernel", "extract"):
        if k in name:
            return k
    return name[:40]


def main(d, last_n=40):
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    rows = list(csv.DictReader(open(f, newline="")))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                 for r in rows), key=lambda x: x[0])
    ks = ks[-last_n:]
    t0 = ks[0][0]
    prev_end = {}
    for s, e, n in ks:
        print(f"{(s - t0) / 1e3:10.2f} {(e - t0) / 1e3:10.2f} {(e - s) / 1e3:8.2f}us {n}")
    dig = [(s, e) for s, e, n in ks if "digest" in n or "build_step" in n]
    gaps = [b[0] - a[1] for a, b in zip(dig, dig[1:])]
    per = [b[0] - a[0] for a, b in zip(dig, dig[1:])]
    if gaps:
        print(f"digest: n={len(dig)} mean dur {statistics.mean(e - s for s, e in dig) / 1e3:.2f} us, "
              f"start-to-start {statistics.mean(per) / 1e3:.2f} us, gap median {statistics.median(gaps) / 1e3:.2f} "
              f"us mean {statistics.mean(gaps) / 1e3:.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
