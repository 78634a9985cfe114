set -o pipefail
mkdir -p gpurun_out
for m in fused off fused off; do
timeout -k 10 200 python bench.py --config c5 --pipeline $m --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/c5_$m.json 2> gpurun_out/c5_$m.err || { tail -30 gpurun_out/c5_$m.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5_$m.json'));print('$m', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'])"
done
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --rccl-selftest --config c5 --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/rccl1_c5.json 2> gpurun_out/rccl1_c5.err || { tail -30 gpurun_out/rccl1_c5.err; exit 1; }
grep "^{" gpurun_out/rccl1_c5.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('rccl1', d['value'], d['ms_per_step'], d['parity'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 1 --rehearse --config c5 --no-e2e > gpurun_out/rehearse_c5_2.json 2> gpurun_out/rehearse_c5_2.err || { tail -30 gpurun_out/rehearse_c5_2.err; exit 1; }
grep "^{" gpurun_out/rehearse_c5_2.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('rehearse2', d['value'], d['parity'])"
