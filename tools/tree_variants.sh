set -o pipefail
mkdir -p gpurun_out
for g in 1 4; do
  echo "groups=$g"
  MDE_TREE_GROUPS=$g timeout -k 10 120 python tools/microbench.py tree > gpurun_out/mb_g$g.log 2>&1 || { tail gpurun_out/mb_g$g.log; exit 1; }
  grep '"B": 64' gpurun_out/mb_g$g.log
done
