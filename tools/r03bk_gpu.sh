#!/bin/bash
# r03bk: digest / tree phase split of one-partition small builds (probe -DMDE_SMALL_PROF), B = 64, 1,000.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bk
mkdir -p $O; rm -rf $O/*
for B in 64 1000; do
  MDE_LIBRARY=tools/ab/libmde_sprof.so timeout -k 10 120 python3 tools/call_trace.py $B 1000 30 1 build > $O/sprof_b$B.log 2>&1 || { tail -5 $O/sprof_b$B.log; exit 1; }
  echo "B=$B"; grep small_prof $O/sprof_b$B.log | tail -4
done
