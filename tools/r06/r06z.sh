# Long build fuzz on the final tree: 8 seeds x 1,000 random shapes (every entry point incl. the
# pipelined whole-workgroup trees and rec8), against the C oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
for s in 71 72 73 74 75 76 77 78; do
  MDE_FUZZ_SEED=$s MDE_FUZZ_CASES=1000 timeout -k 10 300 python -u -m pytest -x -q -s -m gpu -p no:cacheprovider \
    --timeout 280 --timeout-method thread tests/test_fuzz.py >> gpurun_out/r06z_build_fuzz.log 2>&1 || exit 1
done
