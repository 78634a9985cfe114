#!/bin/bash
# r03ab (final tree of the round so far): GPU suite (incl. the full-size BASELINE config tests), default bench, 1-rank RCCL self-test
# (strong C4 + per-build gather run), C5 bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r03ab_pytest.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r03ab_bench.json 2> gpurun_out/r03ab_bench.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --rccl-selftest --no-e2e > gpurun_out/r03ab_selftest.json 2> gpurun_out/r03ab_selftest.err &&
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r03ab_c5.json 2> gpurun_out/r03ab_c5.err &&
timeout -k 10 300 python bench.py --config c3 --profile > gpurun_out/r03ab_c3.json 2> gpurun_out/r03ab_c3.err&&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03ab_smoke.txt 2>&1 &&
timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > gpurun_out/r03ab_batch_bench.jsonl 2> gpurun_out/r03ab_batch_bench.err
