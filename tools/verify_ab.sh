# Verify-step A/B on one box: GPU suite, then tools/microbench.py verify with the tree's libmde.so
# and tools/ab/libmde_ref.so (previous source), alternating, then in-kernel phase times
# (tools/ab/libmde_prof.so, a -DMDE_VERIFY_PROF build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do for lib in ref new; do
  if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
  timeout -k 10 200 python -u tools/microbench.py verify > gpurun_out/vab_${lib}_${rep}.jsonl 2> gpurun_out/vab.err || { tail gpurun_out/vab.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/vab_${lib}_${rep}.jsonl
done; done
MDE_LIBRARY=tools/ab/libmde_prof.so timeout -k 10 200 python -u tools/verify_phase_probe.py > gpurun_out/vprof.log 2>&1 || { tail gpurun_out/vprof.log; exit 1; }
