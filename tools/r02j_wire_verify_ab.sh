set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wire.py tests/test_verify.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02j_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r02j_pytest.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do for lib in ref new; do
  if [ $lib = ref ]; then export MDE_LIBRARY=tools/ab/libmde_ref.so; else unset MDE_LIBRARY; fi
  timeout -k 10 200 python -u tools/microbench.py verify > gpurun_out/r02j_vab_${lib}_${rep}.jsonl 2> gpurun_out/r02j_vab.err || { tail gpurun_out/r02j_vab.err; exit 1; }
done; done
unset MDE_LIBRARY
timeout -k 10 300 python bench.py > gpurun_out/r02j_bench.json 2> gpurun_out/r02j_bench.err || { tail gpurun_out/r02j_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r02j_bench.json').read().splitlines()[-1]);print(d['value'], d['roofline']['frac'], d['parity'])"
# N>1 path with the weak-scaling default: 2 ranks sharing the GPU (gloo), then real RCCL at 1 rank
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 5 --warmup 1 --rehearse --no-e2e > gpurun_out/r02j_rehearse2.json 2> gpurun_out/r02j_rehearse2.err || { tail -30 gpurun_out/r02j_rehearse2.err; exit 1; }
grep '^{' gpurun_out/r02j_rehearse2.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('rehearse2', d['n_gpus'], d['scaling'], d['value'], d['config']['n_partitions'], d['config']['partitions_per_gpu'], d['parity'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 1 --steps 10 --warmup 2 --rccl-selftest --no-e2e --no-cpu-baseline > gpurun_out/r02j_rccl1.json 2> gpurun_out/r02j_rccl1.err || { tail -30 gpurun_out/r02j_rccl1.err; exit 1; }
grep '^{' gpurun_out/r02j_rccl1.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('rccl1', d['n_gpus'], d['scaling'], d['value'], d['parity'])"
