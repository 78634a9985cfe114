set -o pipefail
cd $GRAFT_REPO_ROOT
for shape in 100000000,1000,8,8 10000000,1000,1024,8 100000000,1000,8,1; do
  for r in 1 2; do
    for f in packed wide2 whole; do
      MDE_STEP_TREES=$f MDE_AB_SHAPE=$shape MDE_AB_VARIANT=21 timeout -k 10 120 python tools/prod_ab.py $f 3 40 >> gpurun_out/r06g_ab.jsonl 2>&1 || exit 1
    done
  done
done
