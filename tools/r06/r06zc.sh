# The group tests after the host-pointer paths' early-return drain (StreamDrain).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 250 --timeout-method thread \
  tests/test_group.py -k "not bench" > gpurun_out/r06zc_group.log 2>&1
