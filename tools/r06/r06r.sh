# The production-shape digest alone after an idle spell (tools/idle_probe.py), and the full default
# bench line (CPU baseline, end to end, production shape) as the driver runs it.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/idle_probe.py 10 > gpurun_out/r06r_idle.jsonl 2> gpurun_out/r06r_idle.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/r06r_bench.json 2> gpurun_out/r06r_bench.err
