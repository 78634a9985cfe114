#!/bin/bash
# r03bb: split-schedule trees (tree_body_duo). GPU suite + smoke with them on (the default), then
# kernel traces of one-partition calls, build (small_build_kernel) and tree alone (tree_kernel /
# tree_duo_kernel), B = 64 and 1,000, MDE_TREE_DUO=0 (previous form) vs 1, alternating; batched
# one-partition builds at 10 callers, B = 1,000, both forms.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bb
mkdir -p $O; rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
for rep in 1 2; do
for duo in 0 1; do
for cfg in "64 build" "1000 build" "64 tree" "1000 tree"; do
  set -- $cfg
  d=$O/${2}_b$1_duo${duo}_r$rep
  MDE_TREE_DUO=$duo timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $1 1000 200 1 $2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "duo=$duo rep=$rep $(grep us_per_call $d.log)"
done
done
done
for duo in 0 1; do
  d=$O/batch_b1000_c10_duo$duo
  MDE_TREE_DUO=$duo timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $d -o run -- tests/cpp/build/batch_bench 0.2 1000 10 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "duo=$duo"; grep -h "partitions_per_s\|oracle" $d.log
done
