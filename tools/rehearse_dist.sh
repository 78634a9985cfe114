# N>1 bench rehearsal on a one-GPU box (ranks share cuda:0, gloo gather). Not a measurement.
set -o pipefail
mkdir -p gpurun_out
for cfg in c4 c5; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
    bench.py --gpus 2 --steps 5 --warmup 1 --rehearse --config $cfg > gpurun_out/rehearse_$cfg.json 2> gpurun_out/rehearse_$cfg.err || { tail -30 gpurun_out/rehearse_$cfg.err; exit 1; }
  grep '^{' gpurun_out/rehearse_$cfg.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg', d['n_gpus'], d['value'], d['config']['partitions_per_gpu'], d['parity'])"
done
