#!/bin/bash
# r03bu: per-GPU shard of the strong-scaling C4 run at N = 2, 4, 8 on the final tree
# (bench.py --simulate-world N: rank 0's shard alone, a per-GPU prediction, no collective).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bu
mkdir -p $O; rm -rf $O/*
for n in 1 2 4 8; do
  timeout -k 10 300 python bench.py --simulate-world $n --no-cpu-baseline --no-e2e --no-production-shape --steps 40 > $O/shard_$n.json 2> $O/shard_$n.err || { tail -20 $O/shard_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/shard_$n.json')); print($n, d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['all_ranks_ok'])"
done
