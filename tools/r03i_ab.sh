#!/bin/bash
# r03i: tree top-level priority probe (tools/ab/libmde_topprio3.so) vs the tree's library,
# alternating processes: fused builds on ts8k, c4k, c4, c4/8.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in base topprio3; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python tools/microbench.py pieces:d:ts8k,c4k,c4,c4/8 > gpurun_out/r03i_$lib$rep.jsonl 2> gpurun_out/r03i.err || { tail gpurun_out/r03i.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r03i_$lib$rep.jsonl
done; done
