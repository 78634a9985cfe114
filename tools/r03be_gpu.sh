#!/bin/bash
# r03be: split-schedule trees in the fused build step (one partition per tree workgroup, B > 128 with
# >= 512 partitions). GPU suite, then MDE_TREE_DUO=0/1 A/B of the production shape (8-byte
# timestamps, B = 1,000; tools/prod_shape.py warm) and of fused builds at C4 B = 1,000 layouts A/B;
# small-build digest loads: 4 buckets at a time (tree) vs one (probe library MDE_SMALL_ROUNDS=1).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03be
mkdir -p $O; rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for duo in 0 1; do
  MDE_TREE_DUO=$duo timeout -k 10 200 python tools/prod_shape.py warm > $O/prod_duo${duo}_r$rep.log 2>&1 || { tail -5 $O/prod_duo${duo}_r$rep.log; exit 1; }
  echo "duo=$duo rep=$rep"; cat $O/prod_duo${duo}_r$rep.log | grep fused_us
  for sh in c4k c4bk; do
    MDE_TREE_DUO=$duo timeout -k 10 200 python tools/microbench.py fusedonly:$sh:20 > $O/fused_${sh}_duo${duo}_r$rep.log 2>&1 || { tail -5 $O/fused_${sh}_duo${duo}_r$rep.log; exit 1; }
    echo "duo=$duo rep=$rep $sh $(python3 -c "import json; print(json.load(open('gpurun_out/microbench.json'))['fusedonly'])")"
  done
done
done
for rep in 1 2; do
for lib in new rounds1; do
  for B in 64 1000; do
    d=$O/small_${lib}_b${B}_r$rep
    if [ $lib = rounds1 ]; then export MDE_LIBRARY=tools/ab/libmde_rounds1.so; else unset MDE_LIBRARY; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $B 1000 200 1 build > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  done
done
done
unset MDE_LIBRARY
