#!/bin/bash
# r03bw: record-parallel small-build digest phase for fixed strides vs the bucket loop (probe library -DMDE_SMALL_BUCKET_LOOP)
# (tools/ab/libmde_ref.so): GPU suite, one-partition build / tree kernel traces at B = 64, 1,000,
# alternating, and the production shape.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bw
mkdir -p $O; rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for lib in ref new; do
  if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
  for what in build tree; do
  for B in 64 1000; do
    d=$O/${what}_${lib}_b${B}_r$rep
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $B 1000 200 1 $what > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  done
  done
  timeout -k 10 200 python tools/prod_shape.py warm > $O/prod_${lib}_r$rep.log 2>&1 || { tail -5 $O/prod_${lib}_r$rep.log; exit 1; }
  echo "$lib rep=$rep $(grep -o '"fused_us": [0-9.]*' $O/prod_${lib}_r$rep.log | tr '\n' ' ')"
done
done
unset MDE_LIBRARY
