#!/bin/bash
# r03k: the fused step's wide trees (two waves per partition, B > 128, >= 512 partitions) beside the
# rec8 stream: tree waves at s_setprio 2 / 3 (probe libs) and the dispatch with the tree work
# compiled out (skip: wrong roots, timing only) vs the tree's library, alternating processes.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in base prio2 prio3 skip; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python tools/microbench.py pieces:d:ts8k,c4k,v64k > gpurun_out/r03k_$lib$rep.jsonl 2> gpurun_out/r03k.err || { tail gpurun_out/r03k.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r03k_$lib$rep.jsonl
done; done
