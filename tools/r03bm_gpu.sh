#!/bin/bash
# r03bm: encoders assemble the EpochTreeObject in LDS and store it with 16-byte vector stores
# (the persisted object goes straight to pinned host memory). GPU suite, verify call traces,
# batched verify at 10 callers, standalone encode microbench.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03bm
mkdir -p $O; rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for lib in ref new; do
  if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
  for B in 64 1000; do
    d=$O/verify_${lib}_b${B}_r$rep
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/call_trace.py $B 1000 200 1 verify > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  done
done
done
unset MDE_LIBRARY
for B in 1000 64; do
  f=$O/b${B}_c10_verify.log
  timeout -k 10 60 tests/cpp/build/batch_bench 0.3 $B 10 verify_percall > $f 2>&1 || { tail -5 $f; exit 1; }
  timeout -k 10 60 tests/cpp/build/batch_bench 0.3 $B 10 verify_batched >> $f 2>&1 || { tail -5 $f; exit 1; }
  grep -h partitions_per_s $f
done
