#!/bin/bash
# r03ba: re-check of the restored tree (GPU suite, smoke) and a kernel-trace baseline of one-partition
# calls: build (small_build_kernel) vs tree alone (tree_kernel) at B = 64 and 1,000.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r03ba; rm -rf gpurun_out/r03ba/*
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
  > gpurun_out/r03ba/pytest.log 2>&1 || { tail -20 gpurun_out/r03ba/pytest.log; exit 1; }
tail -2 gpurun_out/r03ba/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ba/smoke.txt 2>&1 || exit 1
for cfg in "64 build" "1000 build" "64 tree" "1000 tree"; do
  set -- $cfg
  d=gpurun_out/r03ba/$2_b$1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $1 1000 200 1 $2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  grep us_per_call $d.log
done
# batched one-partition builds at 10 callers, B = 1,000: kernel + copy trace (are concurrent batches slower per kernel?)
d=gpurun_out/r03ba/batch_b1000_c10
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $d -o run -- tests/cpp/build/batch_bench 0.2 1000 10 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
grep partitions_per_s $d.log
