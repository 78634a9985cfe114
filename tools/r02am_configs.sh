# Round-2 evidence for every BASELINE config on the final kernels: rocprofv3 trace + FETCH/WRITE PMC
# of C2, C3, C4 at B = 1000, C4 layout B, then config 5 (build both replicas + diff + extract),
# fused and unfused, and the 1-rank RCCL self-test of config 5.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r02am}
for spec in "c2 c2" "c3 c3" "c4k c4k" "c4 c4_b --layout b"; do
  bash tools/profile.sh $TAG $spec || exit 1
  echo "profiled $spec"
done
bash tools/c5_check.sh || exit 1
