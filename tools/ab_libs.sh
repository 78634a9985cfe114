# A/B of several engine builds on one box, alternating processes (bench.py, fused default):
#   LIBS="base last:tools/ab/libmde_last.so" ARGS="" bash tools/ab_libs.sh
# "base" = the tree's own libmde.so. Prints ms per step and kernel ms for N=1 and the N=8 shard.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for spec in ${LIBS}; do for sw in 0 8; do
  name=${spec%%:*}
  if [ "$name" = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=${spec#*:}; fi
  timeout -k 10 120 python bench.py --simulate-world $sw ${ARGS:-} --no-cpu-baseline --no-e2e --steps 50 > gpurun_out/abl.json 2>gpurun_out/abl.err || { tail gpurun_out/abl.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abl.json'));print('rep $rep $name shard $sw', d['ms_per_step'], d['roofline']['kernel_ms'], d['parity']['all_ranks_ok'])"
done; done; done
