#!/bin/bash
# r03bf: fused build step at the production shape (ts8k: 8-byte timestamps, B = 1,000), tree /
# stream wave start-end stamps (probe library -DMDE_STEP_STAMPS), MDE_TREE_DUO=0/1 alternating.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bf
mkdir -p $O; rm -rf $O/*
export MDE_LIBRARY=tools/ab/libmde_stamps.so
for rep in 1 2 3; do
for duo in 0 1; do
  MDE_TREE_DUO=$duo timeout -k 10 200 python tools/microbench.py stamps:ts8k > $O/stamps_duo${duo}_r$rep.log 2>&1 || { tail -5 $O/stamps_duo${duo}_r$rep.log; exit 1; }
  python3 - $duo $rep <<'PY'
import json, sys, statistics
rows = json.load(open("gpurun_out/microbench.json"))["stamps"]
m = lambda k: round(statistics.median(r[k] for r in rows), 2)
print("duo", sys.argv[1], "rep", sys.argv[2], {k: m(k) for k in ("tree_start_us", "tree_end_us", "stream_end_us")})
PY
done
done
