#!/bin/bash
# r03bc: batcher host-side phase times (MDE_BATCH_PROFILE=1) for batched builds / verifies at
# B = 1,000 and 64, 1 / 10 / 100 callers; kernel + copy trace of the 10-caller batched build alone.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03bc
mkdir -p $O; rm -rf $O/*
for B in 1000 64; do
for c in 1 10 100; do
for m in batched verify_batched; do
  MDE_BATCH_PROFILE=1 timeout -k 10 60 tests/cpp/build/batch_bench 0.3 $B $c $m > $O/b${B}_c${c}_$m.log 2>&1 || { tail -5 $O/b${B}_c${c}_$m.log; exit 1; }
  echo "B=$B callers=$c $m"; grep -h "partitions_per_s\|batcher_profile" $O/b${B}_c${c}_$m.log
done
done
done
d=$O/trace_b1000_c10_batched
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $d -o run -- tests/cpp/build/batch_bench 0.2 1000 10 batched > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
# small build after the digest-phase change (compare r03bb: 53.2 / 29.0 us with duo trees)
for B in 64 1000; do
  d=$O/build_b$B
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $B 1000 200 1 build > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  grep us_per_call $d.log
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
