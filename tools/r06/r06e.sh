set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in 15 19 21; do
    MDE_AB_VARIANT=$v timeout -k 10 120 python tools/prod_ab.py lib 3 40 >> gpurun_out/r06e_ab.jsonl 2>&1 || exit 1
  done
done
