# Fused build step: tree waves' s_setprio beside the streaming waves (which run at 2): the product
# (`base`, trees at 0) vs probe builds with the trees at 2 (`prio2`) and 3 (`prio3`)
# (tools/build_probe_lib.sh prioN -DMDE_STEP_TREE_PRIO=N, an `s_setprio` at the top of step_trees;
# the switch was removed after the run). Alternating processes, 3 repetitions.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in base prio2 prio3; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 150 python tools/microbench.py pieces:d:${SHAPES:-ts8k,v64k,c4k,c4k/8,ts8,c4,c4/8} > gpurun_out/treeprio.log 2>&1 || { tail gpurun_out/treeprio.log; exit 1; }
  grep '"shape"' gpurun_out/treeprio.log | sed "s/^{/{\"rep\": $rep, \"lib\": \"$lib\", /"
done; done
