#!/bin/bash
# r03bn: fused build step with two trees per tree workgroup (tree_body_pair; MDE_STEP_PAIR=1) vs the
# split-schedule one-tree workgroups (default): parity of the fused-step tests under the switch,
# then the production shape (tools/prod_shape.py warm) and C4 at B = 1,000, alternating.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bn
mkdir -p $O; rm -rf $O/*
MDE_STEP_PAIR=1 timeout -k 10 400 python -u -m pytest tests/test_pipeline.py -m gpu -x -q -k "fused_step or pair_trees or default_variant" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for pair in 0 1; do
  MDE_STEP_PAIR=$pair timeout -k 10 200 python tools/prod_shape.py warm > $O/prod_pair${pair}_r$rep.log 2>&1 || { tail -5 $O/prod_pair${pair}_r$rep.log; exit 1; }
  echo "pair=$pair rep=$rep"; grep fused_us $O/prod_pair${pair}_r$rep.log
  MDE_STEP_PAIR=$pair timeout -k 10 200 python tools/microbench.py fusedonly:c4k:20 > $O/c4k_pair${pair}_r$rep.log 2>&1 || { tail -5 $O/c4k_pair${pair}_r$rep.log; exit 1; }
  echo "pair=$pair rep=$rep c4k $(python3 -c "import json; print(json.load(open('gpurun_out/microbench.json'))['fusedonly'])")"
done
done
