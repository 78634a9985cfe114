# Digest-kernel variant sweep (MDE_DIGEST_VARIANT x MDE_DIGEST_BLOCKS_PER_CU), C4 at N=1 and the N=8 shard.
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3 4 5 6; do
  for cap in 0 ${CAPS:-}; do
    echo "variant=$v cap=$cap"
    MDE_DIGEST_VARIANT=$v MDE_DIGEST_BLOCKS_PER_CU=$cap timeout -k 10 120 python tools/microbench.py digest:1,8 > gpurun_out/sweep_${v}_${cap}.log 2>&1 || { tail -5 gpurun_out/sweep_${v}_${cap}.log; exit 1; }
    grep '"digest"' gpurun_out/sweep_${v}_${cap}.log | python -c "import sys,json; [print(' world', d['world'], 'GBps', d['GBps'], 'digest_us', d['digest_us'], 'build_us', d['build_us']) for d in map(json.loads, sys.stdin)]"
  done
done
