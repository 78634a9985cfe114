# The bench-driven GPU tests on the final bench.py (production shape first, 20 builds per run).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 280 --timeout-method thread \
  tests/test_bench_contract.py tests/test_group.py -k "bench or contract or scaling or torchrun" > gpurun_out/r06zb_bench_tests.log 2>&1
