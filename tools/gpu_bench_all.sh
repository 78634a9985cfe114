# 1-GPU bench of every config (run on the GPU box from the repo root).
set -o pipefail
mkdir -p gpurun_out
for c in ${CONFIGS:-c4 c5 c2 c3}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 ${EXTRA:---no-cpu-baseline} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'])"
done
