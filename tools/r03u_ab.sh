#!/bin/bash
# r03u: host-io tests (direct vs copied outputs), then batcher leaders spinning (default) vs
# sleeping (MDE_BATCH_BLOCKING_SYNC=1) on their batch's event, alternating, 3 repetitions.
set -o pipefail
mkdir -p gpurun_out/r03u; rm -rf gpurun_out/r03u/*
timeout -k 10 200 python -u -m pytest tests/test_host_io.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03u/pytest.log 2>&1 || { tail -30 gpurun_out/r03u/pytest.log; exit 1; }
tail -1 gpurun_out/r03u/pytest.log
for rep in 1 2 3; do for d in 0 1; do
  MDE_BATCH_BLOCKING_SYNC=$d timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > gpurun_out/r03u/b${d}_$rep.jsonl 2>> gpurun_out/r03u/err || exit 1
done; done
