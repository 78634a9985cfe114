set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_bench_contract.py > gpurun_out/r06l_contract.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r06l_bench.json 2> gpurun_out/r06l_bench.err
