#!/bin/bash
# r03p: rec8 with three steps in flight (probe lib tools/ab/libmde_d3.so, -DMDE_REC8_DEPTH=3) vs
# the tree's library (two), alternating processes, 3 repetitions: 8-byte values at B = 1,000 and 64.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in base d3; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python tools/microbench.py pieces:d:ts8k,ts8 > gpurun_out/r03p_$lib$rep.jsonl 2> gpurun_out/r03p.err || { tail gpurun_out/r03p.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r03p_$lib$rep.jsonl
done; done
