#!/bin/bash
# r03b: batcher parity (C program + Python threads) and the production-shape timing
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_batch.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03b_pytest.log 2>&1 &&
timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > gpurun_out/r03b_batch_bench.jsonl 2> gpurun_out/r03b_batch_bench.err
