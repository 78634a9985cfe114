#!/bin/bash
# r03bp: tree node outputs with nontemporal stores (probe library -DMDE_NT_OUT) vs regular stores:
# fused-step parity under the probe, production shape and C4 at B = 1,000, alternating.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bp
mkdir -p $O; rm -rf $O/*
MDE_LIBRARY=tools/ab/libmde_ntout.so timeout -k 10 400 python -u -m pytest tests/test_pipeline.py tests/test_duo_trees.py -m gpu -x -q -k "fused_step or pair_trees or default_variant or duo" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
for lib in new ntout; do
  if [ $lib = ntout ]; then export MDE_LIBRARY=tools/ab/libmde_ntout.so; else unset MDE_LIBRARY; fi
  timeout -k 10 200 python tools/prod_shape.py warm > $O/prod_${lib}_r$rep.log 2>&1 || { tail -5 $O/prod_${lib}_r$rep.log; exit 1; }
  echo "$lib rep=$rep $(grep -o '"fused_us": [0-9.]*' $O/prod_${lib}_r$rep.log | tr '\n' ' ')"
  timeout -k 10 200 python tools/microbench.py fusedonly:c4k:20 > $O/c4k_${lib}_r$rep.log 2>&1 || { tail -5 $O/c4k_${lib}_r$rep.log; exit 1; }
  echo "$lib rep=$rep c4k $(python3 -c "import json; print(json.load(open('gpurun_out/microbench.json'))['fusedonly']['fused_us_per_build'])")"
done
done
unset MDE_LIBRARY
