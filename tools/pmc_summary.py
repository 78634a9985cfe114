"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel, the mean of each counter
per dispatch (every dispatch of that kernel in the file), plus per-4-KiB-step rates when the
workload bytes are given.

    python tools/pmc_summary.py <out.json> <label>=<bytes>=<dir> [...]
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def summarise(d: Path):
    per = defaultdict(lambda: defaultdict(list))
    for f in d.rglob("*counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name") or row.get("Kernel-Name") or "?"
            name = row.get("Counter_Name") or row.get("Counter-Name")
            val = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
            disp = row.get("Dispatch_Id") or row.get("Dispatch-Id") or "0"
            per[k][name].append((disp, val))
    out = {}
    for k, cs in per.items():
        res = {}
        for name, vals in cs.items():
            by = defaultdict(float)
            for disp, v in vals:
                by[disp] += v  # one dispatch may report per-XCD / per-SE rows
            res[name] = sum(by.values()) / len(by)
        out[k] = res
    return out


def main():
    dst = Path(sys.argv[1])
    res = []
    for arg in sys.argv[2:]:
        label, nbytes, d = arg.split("=", 2)
        for k, cs in summarise(Path(d)).items():
            if "digest" not in k and "step" not in k:
                continue
            e = {"label": label, "kernel": k[:120], "counters_per_launch": {n: round(v) for n, v in sorted(cs.items())}}
            steps = int(nbytes) / 4096
            for n, key in (("SQ_INSTS_VALU", "valu_per_4KiB_step"), ("SQ_INSTS_SALU", "salu_per_step"),
                           ("SQ_INSTS_LDS", "lds_per_step")):
                if n in cs:
                    e[key] = round(cs[n] / steps, 2)
            if "FETCH_SIZE" in cs:  # KiB; x 2 on gfx950 (MI355X_MICROARCH.md, HBM section)
                e["hbm_read_bytes"] = round(cs["FETCH_SIZE"] * 1024 * 2)
                e["read_over_algorithmic"] = round(e["hbm_read_bytes"] / int(nbytes), 4)
            if "WRITE_SIZE" in cs:
                e["hbm_write_bytes"] = round(cs["WRITE_SIZE"] * 1024)
            res.append(e)
    dst.write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1)[:4000])


if __name__ == "__main__":
    main()
