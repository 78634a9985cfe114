set -o pipefail
cd $GRAFT_REPO_ROOT
for shape in 100000000,64,8,1 100000000,1000,8,8 20000000,1000,64,1; do
  for r in 1 2; do
    for v in 15 21; do
      MDE_AB_SHAPE=$shape MDE_AB_VARIANT=$v timeout -k 10 120 python tools/prod_ab.py lib 3 40 >> gpurun_out/r06f_ab.jsonl 2>&1 || exit 1
    done
  done
done
for r in 1 2; do
  for v in 16 22; do
    MDE_AB_VARIANT=$v timeout -k 10 120 python tools/prod_ab.py lib 3 40 >> gpurun_out/r06f_ab.jsonl 2>&1 || exit 1
  done
done
