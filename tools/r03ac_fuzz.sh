#!/bin/bash
# r03ac: build fuzz (4 seeds x 200 cases, host / device / pipelined / layout B entry points; the
# host path covers the small one-launch build with LDS sums and the write-once outputs) and the
# batcher's concurrent-caller test at larger sizes.
set -o pipefail
mkdir -p gpurun_out/r03ac; rm -rf gpurun_out/r03ac/*
for seed in 11 12 13 14; do
  MDE_FUZZ_SEED=$seed MDE_FUZZ_CASES=200 timeout -k 10 300 python -u -m pytest tests/test_fuzz.py -m gpu -q --timeout 280 --timeout-method thread > gpurun_out/r03ac/fuzz_$seed.log 2>&1 || { tail -20 gpurun_out/r03ac/fuzz_$seed.log; exit 1; }
  tail -1 gpurun_out/r03ac/fuzz_$seed.log
done
timeout -k 10 300 tests/cpp/build/batch_test 16 60 > gpurun_out/r03ac/batch_16x60.json 2>&1 && tail -1 gpurun_out/r03ac/batch_16x60.json
timeout -k 10 300 tests/cpp/build/batch_test 64 10 > gpurun_out/r03ac/batch_64x10.json 2>&1 && tail -1 gpurun_out/r03ac/batch_64x10.json
