# Two default lines after production_shape's reps 10 -> 20 (steadier difference of two runs).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > gpurun_out/r06x_bench1.json 2> gpurun_out/r06x_bench1.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/r06x_bench2.json 2> gpurun_out/r06x_bench2.err
