# C4 at the reference's default B = 1,000: fused pipeline vs the tree kernel on a second stream
# (now the pair-shape tree kernel for >= 512 partitions), N = 1 and the N = 8 shard
# (--simulate-world 8), alternating processes, 2 repetitions.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for sw in 0 8; do for m in fused streams; do
  timeout -k 10 200 python bench.py --config c4k --pipeline $m --simulate-world $sw --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/c4k_$m.json 2> gpurun_out/c4k_$m.err || { tail -20 gpurun_out/c4k_$m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c4k_$m.json'));print(json.dumps({'rep': $rep, 'sim_world': $sw, 'mode': '$m', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': all(v for v in d['parity'].values() if isinstance(v, bool))}))"
done; done; done
