#!/bin/bash
# r03r: write-once outputs stored straight into pinned staging by the kernels (packed host calls):
# GPU suite, then one-partition build / verify call latency with MDE_DIRECT_OUT=1 (default) vs 0,
# alternating, and one traced B = 1,000 verify run.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03r; rm -rf gpurun_out/r03r/*
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03r/pytest.log 2>&1 || { tail -30 gpurun_out/r03r/pytest.log; exit 1; }
tail -1 gpurun_out/r03r/pytest.log
for rep in 1 2; do for d in 1 0; do for what in build verify; do for B in 64 1000; do
  MDE_DIRECT_OUT=$d timeout -k 10 60 python3 tools/call_trace.py $B 1000 500 1 $what 2>/dev/null | sed "s/^/direct=$d /"
done; done; done; done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03r/v1000 -o run -- python3 tools/call_trace.py 1000 1000 200 1 verify > gpurun_out/r03r/v1000.log 2>&1
