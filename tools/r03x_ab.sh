#!/bin/bash
# r03x: rec8 range bounds in SGPRs (the tree's library) vs HEAD before it (tools/ab/libmde_ref.so),
# alternating processes, 3 repetitions: ts8k, ts8.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in new ref; do
  if [ $lib = new ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python tools/microbench.py pieces:d:ts8k,ts8 > gpurun_out/r03x_$lib$rep.jsonl 2> gpurun_out/r03x.err || { tail gpurun_out/r03x.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r03x_$lib$rep.jsonl
done; done
