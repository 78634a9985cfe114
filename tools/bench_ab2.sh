# Same-box A/B of bench.py flag sets: bash tools/bench_ab2.sh "label1:flags1" "label2:flags2" ...
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  lab=${spec%%:*}; flags=${spec#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 30 $flags > gpurun_out/ab_$lab.json 2> gpurun_out/ab_$lab.err || { tail -5 gpurun_out/ab_$lab.err; exit 1; }
  grep '^{' gpurun_out/ab_$lab.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$lab', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['parity'].get('all_ranks_ok'))"
done
