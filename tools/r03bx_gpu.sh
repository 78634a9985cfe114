#!/bin/bash
# r03bx: final sanity of the committed tree (GPU suite, smoke) and the production call shape
# (batch_bench, 3 repetitions) for stable medians.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bx
mkdir -p $O; rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
grep smoke $O/smoke.txt
for rep in 1 2 3; do
  timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > $O/batch_bench_r$rep.jsonl 2> $O/batch_bench_r$rep.err || { tail -5 $O/batch_bench_r$rep.err; exit 1; }
  tail -1 $O/batch_bench_r$rep.jsonl
done
