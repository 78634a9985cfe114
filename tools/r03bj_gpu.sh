#!/bin/bash
# r03bj: small build takes the buckets' sizes from LDS (digest phase) instead of reloading seg_rec
# in the leaf level. GPU suite, then kernel traces of one-partition builds, new vs the previous
# library (tools/ab/libmde_ref.so), alternating, B = 64 and 1,000.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bj
mkdir -p $O; rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for lib in ref new; do
  for B in 64 1000; do
    d=$O/small_${lib}_b${B}_r$rep
    if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $B 1000 200 1 build > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  done
done
done
unset MDE_LIBRARY
