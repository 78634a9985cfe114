#!/bin/bash
# r03bs: validation of the round's final tree (two-lane padding block included): GPU suite, smoke, default bench line, 1-rank RCCL
# self-test (strong C4 + per-build gather), C5 and C3 bench lines, batch bench (production call
# shape), rocprofv3 trace + FETCH/WRITE PMC of the bench's C4 step.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bs
mkdir -p $O; rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --rccl-selftest --no-e2e > $O/selftest.json 2> $O/selftest.err || { tail -20 $O/selftest.err; exit 1; }
echo selftest ok
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
echo c5 ok
timeout -k 10 300 python bench.py --config c3 --profile > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
echo c3 ok
timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > $O/batch_bench.jsonl 2> $O/batch_bench.err || { tail -20 $O/batch_bench.err; exit 1; }
echo batch ok
bash tools/profile.sh r03bs c4 c4 > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo profile ok
