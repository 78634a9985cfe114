#!/bin/bash
# r03q: timeline of one-partition synchronous builds (kernel + memory-copy trace):
# B = 64 and 1,000 with nodes, 1,000 without nodes, 256 and 512 with nodes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03q; rm -rf gpurun_out/r03q/*
for cfg in "64 1" "1000 1" "1000 0" "256 1" "512 1"; do
  set -- $cfg
  d=gpurun_out/r03q/b$1_n$2
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $1 1000 200 $2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  grep us_per_call $d.log
done
