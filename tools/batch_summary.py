"""Print a table of a batch_bench JSONL file (tests/cpp/batch_bench.c)."""
import json
import sys

for ln in open(sys.argv[1]):
    d = json.loads(ln)
    if "case" in d:
        print(f"{d['case']:15s} P={d['callers']:3d} n={d['records']:6d} B={d['n_buckets']:4d} "
              f"calls/s={d.get('calls_per_s', d.get('partitions_per_s', 0)):10.0f} med={d['latency_median_us']:8.1f} "
              f"p90={d['latency_p90_us']:8.1f} rpb={d.get('mean_requests_per_batch', '')} "
              f"host_comp={d.get('host_compressions_per_call', '')}")
    else:
        print(d)
