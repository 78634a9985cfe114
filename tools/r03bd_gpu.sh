#!/bin/bash
# r03bd: batcher with early leader handoff + per-caller copy-out: batch tests, then A/B of
# MDE_BATCH_EARLY (0 = hand off after the launch) and MDE_BATCH_SLOTS (4 / 8) at B = 1,000 and 64,
# 10 and 100 callers (MDE_BATCH_PROFILE=1 phase times).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bd
mkdir -p $O; rm -rf $O/*
timeout -k 10 300 python -u -m pytest tests/test_batch.py tests/test_concurrency.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for cfg in "1 4" "0 4" "1 8"; do
  set -- $cfg
  for B in 1000 64; do
  for c in 10 100; do
  for m in batched verify_batched; do
    f=$O/e$1_s$2_b${B}_c${c}_${m}_r$rep.log
    MDE_BATCH_EARLY=$1 MDE_BATCH_SLOTS=$2 MDE_BATCH_PROFILE=1 timeout -k 10 60 tests/cpp/build/batch_bench 0.3 $B $c $m > $f 2>&1 || { tail -5 $f; exit 1; }
    echo "early=$1 slots=$2 B=$B callers=$c $m $(grep -h partitions_per_s $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["partitions_per_s"], d["latency_median_us"], d.get("mean_requests_per_batch"))') $(grep -h batcher_profile $f)"
  done
  done
  done
done
done
