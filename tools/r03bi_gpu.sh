#!/bin/bash
# r03bi: phase times inside the fused verify kernel for one-partition calls (probe library
# -DMDE_VERIFY_PROF: wall_clock64 stamps, 100 MHz), B = 64 and 1,000, two peers.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bi
mkdir -p $O; rm -rf $O/*
for B in 64 1000; do
  MDE_LIBRARY=tools/ab/libmde_vprof.so timeout -k 10 120 python3 tools/call_trace.py $B 1000 30 1 verify > $O/vprof_b$B.log 2>&1 || { tail -5 $O/vprof_b$B.log; exit 1; }
  echo "B=$B"; grep verify_prof $O/vprof_b$B.log | tail -5
done
