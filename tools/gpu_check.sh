# GPU parity tests + tree/digest micro-benchmarks (run on the GPU box from the repo root).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/microbench.py ${MB:-tree digest} > gpurun_out/mb.log 2>&1 || { tail -20 gpurun_out/mb.log; exit 1; }
grep kernel gpurun_out/mb.log
