#!/bin/bash
# r03g: layout-B row reduction + verify with on-device local trees: GPU suite, then layout-B A/B
# (fused steps, c4bk/c4b) against the previous library, and the production-shape timing.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03g_pytest.log 2>&1 &&
timeout -k 10 300 python tools/microbench.py pieces:d:c4bk,c4b,ts8k,c4k > gpurun_out/r03g_ab.jsonl 2> gpurun_out/r03g_ab.err &&
timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > gpurun_out/r03g_batch_bench.jsonl 2> gpurun_out/r03g_batch_bench.err
