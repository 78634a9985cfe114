#!/bin/bash
# r03h: A/B of the tree's libmde.so against tools/ab/libmde_ref.so (commit 2452fe0: before the
# layout-B row reduction and the rec8 trim), alternating processes, 3 repetitions:
# fused builds and the digest/binning kernel alone on c4bk, c4b, ts8k.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in ref new; do
  if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
  timeout -k 10 200 python tools/microbench.py pieces:d:c4bk,c4b,ts8k > gpurun_out/r03h_$lib$rep.jsonl 2> gpurun_out/r03h.err || { tail gpurun_out/r03h.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r03h_$lib$rep.jsonl
done; done
