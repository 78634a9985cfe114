# Two more default lines (another box) with the production shape over 20 builds per run.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > gpurun_out/r06y_bench1.json 2> gpurun_out/r06y_bench1.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/r06y_bench2.json 2> gpurun_out/r06y_bench2.err
