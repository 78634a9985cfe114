set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_group.py tests/test_server.py tests/test_integration.py > gpurun_out/r06k_group_server.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_bench_contract.py > gpurun_out/r06k_contract.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r06k_bench.json 2> gpurun_out/r06k_bench.err
