#!/bin/bash
# r03y: rec8 with scalar range bounds (new) vs HEAD before it (ref), and the new kernel with the
# rec8 stream at priority 0 / 1 in the fused step (sp0, sp1), and tree workgroups placed after
# the stream (trlast); alternating processes, 3 repetitions: ts8k, ts8.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in new ref sp0 sp1 trlast; do
  if [ $lib = new ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python tools/microbench.py pieces:d:ts8k,ts8 > gpurun_out/r03y_$lib$rep.jsonl 2> gpurun_out/r03y.err || { tail gpurun_out/r03y.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r03y_$lib$rep.jsonl
done; done
