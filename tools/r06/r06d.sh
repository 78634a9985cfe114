set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in 15 19 21; do
    MDE_AB_VARIANT=$v timeout -k 10 120 python tools/prod_ab.py lib 3 40 >> gpurun_out/r06d_ab.jsonl 2>&1 || exit 1
  done
done
for v in 15 19 21; do
  echo "variant $v" >> gpurun_out/r06d_place.jsonl
  MDE_AB_VARIANT=$v MDE_LIBRARY=tools/abx/libmde_stamps.so timeout -k 10 120 python tools/placement_probe.py 100000000 1000 8 1 >> gpurun_out/r06d_place.jsonl 2>&1 || exit 1
done
