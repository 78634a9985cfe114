set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_group.py -k "multi_build or places_partition" > gpurun_out/r06o_group.log 2>&1 &&
timeout -k 10 120 python tools/prod_ab.py lib 3 40 > gpurun_out/r06n_prodab.jsonl 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-e2e > gpurun_out/r06n_bench.json 2> gpurun_out/r06n_bench.err &&
timeout -k 10 120 python tools/prod_ab.py lib 3 40 >> gpurun_out/r06n_prodab.jsonl 2>&1
