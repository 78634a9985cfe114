# Round check (suite, smoke, bench, rocprofv3 of C4 and of C4 at B = 1000), then the tree kernel
# with fully unrolled SHA-256 rounds (probe build) vs the compact loop, alternating processes.
set -o pipefail
TAG=r02y bash tools/gpu_round.sh || exit 1
bash tools/profile.sh r02y c4k c4k || exit 1
for rep in 1 2; do for lib in base shaunroll; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python -u tools/microbench.py tree > gpurun_out/r02y_tree_$lib.jsonl 2> gpurun_out/r02y_tree.err || { tail gpurun_out/r02y_tree.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r02y_tree_$lib.jsonl
done; done
