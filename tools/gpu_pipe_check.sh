# Full GPU suite + per-shard bench lines for each pipelining mode + a kernel timeline of the
# N=8 shard (run on the GPU box from the repo root).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for w in 8 4 2 1; do
for m in ${MODES:-fused streams}; do
timeout -k 10 120 python bench.py --simulate-world $w --no-cpu-baseline --no-e2e --steps 50 --pipeline $m ${BENCH_ARGS:-} > gpurun_out/f_${w}_$m.json 2>gpurun_out/f_${w}_$m.err || { tail -20 gpurun_out/f_${w}_$m.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/f_${w}_$m.json'));print($w, '$m', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['achieved'], d['parity']['all_ranks_ok'])"
done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlf8 -o run -- python3 bench.py --simulate-world 8 --no-cpu-baseline --no-e2e --steps 50 > gpurun_out/tlf8.json 2> gpurun_out/tlf8.err && python tools/timeline.py gpurun_out/tlf8 6
