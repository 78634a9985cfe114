# What bench's end-to-end leg leaves behind that slows the production-shape digest alone
# (tools/e2e_after_probe.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u tools/e2e_after_probe.py > gpurun_out/r06t_after.jsonl 2> gpurun_out/r06t_after.err
