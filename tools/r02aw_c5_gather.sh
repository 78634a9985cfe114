# Config 5 with the per-partition diff counts gathered beside the roots (N > 1): the C5 check
# (fused / unfused at N = 1, 1-rank RCCL, 2 gloo ranks sharing the GPU), then 2 gloo ranks unfused.
set -o pipefail
mkdir -p gpurun_out
bash tools/c5_check.sh || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 1 --rehearse --config c5 --pipeline off --no-e2e > gpurun_out/rehearse_c5_2_off.json 2> gpurun_out/rehearse_c5_2_off.err || { tail -30 gpurun_out/rehearse_c5_2_off.err; exit 1; }
grep "^{" gpurun_out/rehearse_c5_2_off.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('rehearse2_off', d['value'], d['parity'])"
grep "^{" gpurun_out/rehearse_c5_2.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('rehearse2_fused', d['parity'])"
