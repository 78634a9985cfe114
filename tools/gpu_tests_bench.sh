set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
