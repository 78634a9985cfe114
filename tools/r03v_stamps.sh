#!/bin/bash
# r03v: inside one fused build step (probe lib -DMDE_STEP_STAMPS): when the tree waves and the
# streaming waves start and end, per shape.
set -o pipefail
mkdir -p gpurun_out
export MDE_LIBRARY=tools/ab/libmde_stamps.so
for sh in ts8k c4k v64k c4 c4k/8; do
  timeout -k 10 120 python tools/microbench.py stamps:$sh 2>> gpurun_out/r03v.err || exit 1
done
