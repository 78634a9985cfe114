# Fuzz on the final tree: the build fuzz (tests/test_fuzz.py) at four new seeds x 200 cases, the
# seeded random-shape pipeline / group / service tests, and the long decode + verify fuzz.
set -o pipefail
cd $GRAFT_REPO_ROOT
for s in 61 62 63 64; do
  MDE_FUZZ_SEED=$s MDE_FUZZ_CASES=200 timeout -k 10 300 python -u -m pytest -x -q -m gpu -p no:cacheprovider \
    --timeout 250 --timeout-method thread tests/test_fuzz.py >> gpurun_out/r06w_build_fuzz.log 2>&1 || exit 1
done
timeout -k 10 500 python -u tools/fuzz_long.py 3 20000 300 > gpurun_out/r06w_fuzz_long.jsonl 2> gpurun_out/r06w_fuzz_long.err
