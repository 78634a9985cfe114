# Standalone decode A/B on one box: GPU suite, then tools/microbench.py decode with the tree's
# libmde.so and tools/ab/libmde_ref.so (previous source), alternating processes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2; do for lib in ref new; do
  if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
  timeout -k 10 200 python -u tools/microbench.py decode > gpurun_out/dab_${lib}_${rep}.jsonl 2> gpurun_out/dab.err || { tail gpurun_out/dab.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/dab_${lib}_${rep}.jsonl
done; done
timeout -k 10 300 python -u tools/fuzz_long.py 1 5000 50 > gpurun_out/fuzz3.jsonl 2> gpurun_out/fuzz3.err || { tail gpurun_out/fuzz3.err; exit 1; }
cat gpurun_out/fuzz3.jsonl
