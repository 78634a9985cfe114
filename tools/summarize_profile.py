#!/usr/bin/env python3
"""Summarize a tools/profile.sh run (rocprofv3 CSVs) into profiles/<tag>_<cfg>.json and update
profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.

    python tools/summarize_profile.py gpurun_out/prof_r01_c4 r01 c4      (label c4_b for --layout b)

HBM bytes per launch = FETCH_SIZE (KiB) x 1024 x 2: on gfx950 FETCH_SIZE reports exactly half of a
wide coalesced streaming read (MI355X_MICROARCH.md, section HBM).
"""
import csv
import json
import shutil
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def short(name):
    for k in ("build_step_kernel", "bucket_digest_kernel", "tagged_step_kernel", "tagged_digest_kernel", "tree_kernel", "diff_kernel",
              "synth_values_kernel", "synth_tags_kernel", "tag_keys_kernel", "verify_kernel",
              "encode_kernel", "decode_kernel", "extract"):
        if k in name:
            return k
    return name[:60]


def main(src, tag, cfg):
    src = Path(src)
    out = {"tag": tag, "config": cfg, "kernels": {}}
    stats = rows(src / "trace" / "run_kernel_stats.csv")
    for r in stats:
        out["kernels"].setdefault(short(r["Name"]), {
            "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
            "max_ns": float(r["MaxNs"]), "pct": float(r["Percentage"])})
    bench = json.loads([x for x in (src / "bench_trace.json").read_text().splitlines() if x.startswith("{")][-1])
    alg = bench["roofline"]["algorithmic_bytes_per_launch"]
    kern = bench["roofline"].get("kernel", "bucket_digest_kernel").split(" ")[0]
    out["dominant_kernel"] = kern
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = src / f"pmc_{kind}" / "run_counter_collection.csv"
        if not f.exists():
            continue
        vals = [float(r["Counter_Value"]) for r in rows(f)
                if kern in r["Kernel_Name"] and r["Counter_Name"] == counter]
        if vals:
            out[f"digest_{counter}_kib_median"] = statistics.median(vals)
    fk = out.get("digest_FETCH_SIZE_kib_median")
    dk = out["kernels"].get(kern)
    if fk and dk:
        hbm = int(fk * 1024 * 2)
        out["digest_hbm_read_bytes_per_launch"] = hbm
        out["digest_algorithmic_bytes_per_launch"] = alg
        out["digest_traffic_over_algorithmic"] = round(hbm / alg, 4)
        out["digest_achieved_GBps_rocprof_avg"] = round(alg / dk["avg_ns"], 1)
        out["digest_frac_of_8TBps_rocprof_avg"] = round(alg / dk["avg_ns"] / 8000.0, 4)
        out["bench_event_kernel_ms"] = bench["roofline"]["kernel_ms"]
        tfile = ROOT / "profiles" / "pmc_traffic.json"
        t = json.loads(tfile.read_text()) if tfile.exists() else {}
        t[cfg] = {"algorithmic_bytes": alg, "hbm_read_bytes_per_launch": hbm, "source": f"profiles/{tag}_{cfg}.json"}
        tfile.write_text(json.dumps(t, indent=1) + "\n")
    # per-launch durations of the dominant kernel from the trace: the first launch of a process
    # runs on cold TLBs and inflates the stats average of a short run
    tr = list((src / "trace").glob("*kernel_trace.csv"))
    if tr:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows(tr[0])
                if kern in r["Kernel_Name"]]
        if len(durs) > 1:
            k = int(bench.get("steps", 0))
            out["dominant_kernel_trace"] = {
                "launches": len(durs), "first_ns": durs[0],
                "avg_ns_excluding_first": round(statistics.mean(durs[1:]), 1),
                "median_ns": statistics.median(durs)}
            # the bench's K timed launches are the last K (warm-up and calibration launches before)
            if 0 < k <= len(durs):
                out["dominant_kernel_trace"]["avg_ns_timed_launches"] = round(statistics.mean(durs[-k:]), 1)
                out["dominant_kernel_trace"]["timed_launches"] = k
    dst = ROOT / "profiles" / f"{tag}_{cfg}.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    shutil.copy(src / "trace" / "run_kernel_stats.csv", ROOT / "profiles" / f"{tag}_{cfg}_kernel_stats.csv")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
