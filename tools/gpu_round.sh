# One GPU session: full parity suite, smoke, default bench line, rocprofv3 profile of the default
# bench workload (trace + FETCH_SIZE + WRITE_SIZE passes). Run on the GPU box from the repo root:
#   TAG=r01d bash tools/gpu_round.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01d}
bash tools/gpu_tests_bench.sh || exit 1
bash tools/profile.sh $TAG c4 c4 || exit 1
python tools/timeline.py gpurun_out/prof_${TAG}_c4/trace 8
