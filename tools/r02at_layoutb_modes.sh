# Layout B (records in write order + bucket tags) through bench.py: fused pipeline vs the tree
# kernel on a second stream (the N = 1 default), C4 at B = 64 and B = 1,000, N = 1 and the N = 8
# shard (--simulate-world 8), alternating processes, 2 repetitions.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for cfg in c4 c4k; do for sw in 0 8; do for m in fused streams; do
  timeout -k 10 200 python bench.py --config $cfg --layout b --pipeline $m --simulate-world $sw --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/lb_$m.json 2> gpurun_out/lb_$m.err || { tail -20 gpurun_out/lb_$m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lb_$m.json'));print(json.dumps({'rep': $rep, 'config': '$cfg', 'sim_world': $sw, 'mode': '$m', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': all(v for v in d['parity'].values() if isinstance(v, bool))}))"
done; done; done; done
