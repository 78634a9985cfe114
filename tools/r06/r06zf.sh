# The bench-contract tests after the scaling-curve test takes each engine's best of two runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 400 --timeout-method thread \
  tests/test_bench_contract.py > gpurun_out/r06zf_contract.log 2>&1
