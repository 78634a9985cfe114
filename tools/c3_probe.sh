# C3 (64 x 1M x 1 KiB = 65.5 GB) on one box: read-ceiling probes over the same byte count, then
# the bench's C3 line in fused and serial modes. Run on the GPU box from the repo root:
#   TAG=r02b bash tools/c3_probe.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02b}
timeout -k 10 240 tools/readceil 65536000000 > gpurun_out/${TAG}_readceil_c3.jsonl || exit 1
tail -3 gpurun_out/${TAG}_readceil_c3.jsonl
for mode in fused off; do
  timeout -k 10 300 python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    --pipeline $mode ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_c3_$mode.json 2> gpurun_out/${TAG}_bench_c3_$mode.err \
    || { tail -20 gpurun_out/${TAG}_bench_c3_$mode.err; exit 1; }
  cut -c1-400 gpurun_out/${TAG}_bench_c3_$mode.json
done
