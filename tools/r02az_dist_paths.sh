# The N > 1 bench paths on the one-GPU box: 4 gloo ranks sharing the GPU (default C4 workload,
# weak scaling), the 1-rank RCCL self-test, and 2 gloo ranks of config 5; prints each line's
# root_gather description and parity gates.
set -o pipefail
mkdir -p gpurun_out
show() { grep "^{" $1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$2', d['value'], d['config']['root_gather'], d['parity'])"; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --steps 5 --warmup 1 --rehearse --no-e2e > gpurun_out/rehearse4.json 2> gpurun_out/rehearse4.err || { tail -20 gpurun_out/rehearse4.err; exit 1; }
show gpurun_out/rehearse4.json rehearse4
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 1 --rccl-selftest --no-e2e --steps 10 > gpurun_out/rccl1.json 2> gpurun_out/rccl1.err || { tail -20 gpurun_out/rccl1.err; exit 1; }
show gpurun_out/rccl1.json rccl1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29516 bench.py --gpus 2 --steps 5 --warmup 1 --rehearse --config c5 --no-e2e > gpurun_out/rehearse_c5.json 2> gpurun_out/rehearse_c5.err || { tail -20 gpurun_out/rehearse_c5.err; exit 1; }
show gpurun_out/rehearse_c5.json rehearse2_c5
