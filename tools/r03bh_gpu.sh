#!/bin/bash
# r03bh: verify outputs stored once (valid / peer statuses straight into pinned memory, no D2H copy):
# GPU suite, one-partition verify call traces (B = 64, 1,000), batched verify at 10 callers.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bh
mkdir -p $O; rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for B in 64 1000; do
  d=$O/verify_b$B
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $B 1000 200 1 verify > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  grep us_per_call $d.log
done
for rep in 1 2; do
for B in 1000 64; do
  for m in verify_percall verify_batched; do
    f=$O/b${B}_c10_${m}_r$rep.log
    timeout -k 10 60 tests/cpp/build/batch_bench 0.3 $B 10 $m > $f 2>&1 || { tail -5 $f; exit 1; }
    echo "B=$B $m $(grep -h partitions_per_s $f)"
  done
done
done
