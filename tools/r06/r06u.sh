# The default bench line with the production shape measured first (before the CPU baseline and the
# end-to-end leg), twice, and the end-to-end after-effect probe (tools/e2e_after_probe.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > gpurun_out/r06u_bench1.json 2> gpurun_out/r06u_bench1.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/r06u_bench2.json 2> gpurun_out/r06u_bench2.err
