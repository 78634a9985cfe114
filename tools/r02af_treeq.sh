# Fused build step: partitions per packed tree wave (Q) under other caps (probe builds,
# tools/build_probe_lib.sh qN -DMDE_STEP_TREE_QMAX=Nu) vs the tree's own build, on the small
# arenas where the trees' critical path can outlast the stream. Alternating processes, 3 reps.
#   LIBS="base q16" SHAPES=ts8,c4 bash tools/r02af_treeq.sh
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in ${LIBS:-base q2 q4 q8}; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 150 python tools/microbench.py pieces:d:${SHAPES:-ts8,c4/8,c4} > gpurun_out/treeq.log 2>&1 || { tail gpurun_out/treeq.log; exit 1; }
  grep '"shape"' gpurun_out/treeq.log | sed "s/^{/{\"rep\": $rep, \"lib\": \"$lib\", /"
done; done
