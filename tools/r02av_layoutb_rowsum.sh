# Rejected experiment (code reverted after the run): layout B, records >= 1 KiB at B > 64, one
# wave sum + one bin add per 1 KiB row (`base`) vs 64 slot adds sharing 64 / L slots (`head`),
# bench.py C4 at B = 1,000 and B = 64 in layout B, fused, alternating processes, 3 repetitions.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2 3; do for cfg in c4k c4; do for lib in base head; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python bench.py --config $cfg --layout b --pipeline fused --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/lb.json 2> gpurun_out/lb.err || { tail -20 gpurun_out/lb.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lb.json'));print(json.dumps({'rep': $rep, 'config': '$cfg', 'lib': '$lib', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': all(v for v in d['parity'].values() if isinstance(v, bool))}))"
done; done; done
