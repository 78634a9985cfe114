# GPU suite and smoke after every synchronous entry point drains its streams on return.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r06ze_gpu_suite.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06ze_smoke.log 2>&1
