# Same-box A/B of bench.py digest tunings: bash tools/bench_ab.sh "4,2 0,0 4,2 0,0"
set -o pipefail
mkdir -p gpurun_out
for t in $1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --tuning $t ${EXTRA:-} > gpurun_out/ab_$t.json 2> gpurun_out/ab_$t.err || { tail -5 gpurun_out/ab_$t.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$t.json'));print('$t', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])"
done
