# Digest variant A/B (run on the GPU box from the repo root): VARIANTS="7 11" bash tools/ab_variant.sh
# 1) interleaved in one process (standalone digest), 2) fused bench lines per variant, alternating.
set -o pipefail
mkdir -p gpurun_out
V=${VARIANTS:-7 11}
timeout -k 10 400 python tools/microbench.py ab:$(echo $V | tr ' ' ',') > gpurun_out/ab_micro.log 2>&1 || { tail -20 gpurun_out/ab_micro.log; exit 1; }
grep '^{' gpurun_out/ab_micro.log
for rep in 1 2; do for v in $V; do for sw in 0 8; do
  timeout -k 10 120 python bench.py --simulate-world $sw --tuning $v,2 --no-cpu-baseline --no-e2e --steps 50 > gpurun_out/abv_$v_$sw.json 2>gpurun_out/abv.err || { tail gpurun_out/abv.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abv_$v_$sw.json'));print('rep $rep variant $v shard $sw', d['ms_per_step'], d['roofline']['kernel_ms'], d['parity']['all_ranks_ok'])"
done; done; done
