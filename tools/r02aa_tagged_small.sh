# Layout-B small-record path: pipeline + parity tests, then the tree's library vs the previous
# build (tools/ab/libmde_ref.so), alternating processes, on layout-B shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pipeline.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02aa_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02aa_pytest.log; [ $rc = 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r02aa_pytest.log | head -60; exit 1; }
for rep in 1 2; do for lib in ref new; do
  if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
  timeout -k 10 300 python -u tools/microbench.py pieces:d:c4b,c4bk,ts8bk > gpurun_out/r02aa_$lib.jsonl 2> gpurun_out/r02aa.err || { tail gpurun_out/r02aa.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r02aa_$lib.jsonl | cut -c1-220
done; done
