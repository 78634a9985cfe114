# N>1 bench rehearsal on a one-GPU box (ranks share cuda:0, gloo gather). Not a measurement.
set -o pipefail
mkdir -p gpurun_out
for run in "2 c4 5" "3 c4 9" "2 c4 8" "2 c5 3"; do
  set -- $run
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 29512 \
    bench.py --gpus $1 --steps $3 --warmup 1 --rehearse --config $2 --no-e2e > gpurun_out/rehearse_$2_$1.json 2> gpurun_out/rehearse_$2_$1.err || { tail -30 gpurun_out/rehearse_$2_$1.err; exit 1; }
  grep '^{' gpurun_out/rehearse_$2_$1.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$run', d['n_gpus'], d['value'], d['config']['partitions_per_gpu'], d['parity'])"
done
