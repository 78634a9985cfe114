# Round-6 bench lines for the other BASELINE configs on the final library (C2, C3 at 64 GiB,
# C4 at B = 1,000, C5), each with the C-oracle sample check; no CPU baseline / end-to-end legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c2 c3 c4k c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --no-cpu-baseline --no-e2e \
    > gpurun_out/r06p_bench_$c.json 2> gpurun_out/r06p_bench_$c.err || exit 1
done
