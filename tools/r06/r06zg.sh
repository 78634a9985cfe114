# The driver's N = 8 launcher form rehearsed on one GPU: torch.distributed.run with 8 ranks,
# rank 0 driving the 8-member group (--rehearse: every member on GPU 0, copy gather), ranks 1-7
# joining its barriers; C4 and C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c4 c5; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 8 --steps 10 --rehearse --config $c \
    > gpurun_out/r06zg_torchrun8_$c.json 2> gpurun_out/r06zg_torchrun8_$c.err || exit 1
done
