# A/B of two engine builds on one box, alternating processes: the tree's libmde.so vs
# tools/ab/libmde_ref.so (built from the previous source). ARGS = bench flags.
#   ARGS="--layout b --pipeline off" bash tools/ab_lib.sh
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in ref new; do for sw in 0 8; do
  if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
  timeout -k 10 120 python bench.py --simulate-world $sw ${ARGS:-} --no-cpu-baseline --no-e2e --steps 50 > gpurun_out/abl.json 2>gpurun_out/abl.err || { tail gpurun_out/abl.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abl.json'));print('rep $rep $lib shard $sw', d['ms_per_step'], d['roofline']['kernel_ms'], d['parity']['all_ranks_ok'])"
done; done; done
