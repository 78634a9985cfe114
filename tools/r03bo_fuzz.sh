#!/bin/bash
# r03bo: fuzz on the final tree (split-schedule trees, write-once verify outputs, batcher changes):
# build fuzz 4 seeds x 200 cases, long decode/verify fuzz, batcher concurrent-caller tests.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bo
mkdir -p $O; rm -rf $O/*
for seed in 21 22 23 24; do
  MDE_FUZZ_SEED=$seed MDE_FUZZ_CASES=200 timeout -k 10 300 python -u -m pytest tests/test_fuzz.py -m gpu -q --timeout 280 --timeout-method thread > $O/fuzz_$seed.log 2>&1 || { tail -20 $O/fuzz_$seed.log; exit 1; }
  tail -1 $O/fuzz_$seed.log
done
timeout -k 10 400 python -u tools/fuzz_long.py 2 10000 200 > $O/fuzz_long.jsonl 2>&1 || { tail -20 $O/fuzz_long.jsonl; exit 1; }
cat $O/fuzz_long.jsonl | tail -4
timeout -k 10 300 tests/cpp/build/batch_test 16 60 > $O/batch_16x60.json 2>&1 && tail -1 $O/batch_16x60.json
timeout -k 10 300 tests/cpp/build/batch_test 64 10 > $O/batch_64x10.json 2>&1 && tail -1 $O/batch_64x10.json
