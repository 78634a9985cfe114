#!/bin/bash
# r03d: 4-slot batcher, deep-group spill area, shim replay; then the production-shape timing
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_batch.py tests/test_wire.py tests/test_integration.py tests/test_verify.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03d_pytest.log 2>&1 &&
timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > gpurun_out/r03d_batch_bench.jsonl 2> gpurun_out/r03d_batch_bench.err
