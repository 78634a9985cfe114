#!/bin/bash
# r03s: batcher with write-once outputs in pinned memory: batch / shim / verify GPU tests, then
# batch_bench with MDE_DIRECT_OUT=1 (default) and =0.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_batch.py tests/test_integration.py tests/test_verify.py -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03s_pytest.log 2>&1 || { tail -30 gpurun_out/r03s_pytest.log; exit 1; }
tail -1 gpurun_out/r03s_pytest.log
MDE_DIRECT_OUT=1 timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > gpurun_out/r03s_batch_direct.jsonl 2> gpurun_out/r03s_bb.err &&
MDE_DIRECT_OUT=0 timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > gpurun_out/r03s_batch_copy.jsonl 2>> gpurun_out/r03s_bb.err
