# Rejected experiment (code reverted after the run): pipeline depth 3 -- wide trees split over two
# launches via mde_set_pipeline_depth -- vs depth 2, same library, alternating processes, 3 repetitions;
# GPU suite first (depth-3 parity tests, 107/107 at the time).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2 3; do for depth in 2 3; do
  MDE_PIPELINE_DEPTH=$depth timeout -k 10 150 python tools/microbench.py pieces:d:${SHAPES:-ts8k,v64k,c4k,ts8,c4} > gpurun_out/depth3.log 2>&1 || { tail gpurun_out/depth3.log; exit 1; }
  grep '"shape"' gpurun_out/depth3.log | sed "s/^{/{\"rep\": $rep, \"depth\": $depth, /"
done; done
