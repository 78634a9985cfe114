#!/bin/bash
# r03bg: split-schedule tree parity over every shape boundary (tests/test_duo_trees.py); kernel +
# copy trace of one-partition verify calls (B = 64, 1,000).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bg
mkdir -p $O; rm -rf $O/*
timeout -k 10 300 python -u -m pytest tests/test_duo_trees.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for B in 64 1000; do
  d=$O/verify_b$B
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $B 1000 200 1 verify > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  grep us_per_call $d.log
done
