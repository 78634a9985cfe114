#!/bin/bash
# r03m: where C4 at B = 1,000 (layout A) reads its 0.66 % of extra HBM bytes: FETCH_SIZE of the
# digest kernel alone under the automatic choice (window kernel, interleaved pieces), the window
# kernel with one range per wave, round 1's kernel with one range, and the byte kernel in pieces.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m; rm -rf gpurun_out/r03m/*
for s in d v13x x v12d; do
  out=gpurun_out/r03m/c4k_$s
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out -o run -- python3 tools/microbench.py digestonly:c4k:3:$s > $out.log 2>&1 || { tail -5 $out.log; exit 1; }
  grep -h "_us" $out.log | tail -1
done
