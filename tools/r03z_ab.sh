#!/bin/bash
# r03z: rec8 scalar bounds in the standalone kernel only (new) vs HEAD (ref); probes: fused with
# scalar bounds plus s_sleep 1 / 2 per scan step (fscs1, fscs2), fused as shipped plus s_sleep 1
# (s1); alternating processes, 3 repetitions: ts8k, ts8.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in new ref fscs1 fscs2 s1; do
  if [ $lib = new ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python tools/microbench.py pieces:d:ts8k,ts8 > gpurun_out/r03z_$lib$rep.jsonl 2> gpurun_out/r03z.err || { tail gpurun_out/r03z.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r03z_$lib$rep.jsonl
done; done
