#!/bin/bash
# r03bv: does the kernel-argument segment's placement matter for one-partition calls?
# HIP_FORCE_DEV_KERNARG=0 / 1 (kernargs in host / device memory), small-build phase probe and
# kernel traces at B = 64, 1,000.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bv
mkdir -p $O; rm -rf $O/*
for rep in 1 2; do
for kd in 0 1; do
  for B in 64 1000; do
    d=$O/build_k${kd}_b${B}_r$rep
    HIP_FORCE_DEV_KERNARG=$kd timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $B 1000 200 1 build > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    echo "kernarg_dev=$kd B=$B $(grep us_per_call $d.log)"
  done
done
done
