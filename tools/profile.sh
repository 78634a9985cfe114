# rocprofv3 profiles of the bench workload (run on the GPU box from the repo root).
#   bash tools/profile.sh <tag> [config] [label] [extra bench flags...]
#   e.g. bash tools/profile.sh r01c c4 c4_b --layout b
# 1) kernel trace + stats (bench's default warm-up: the timed launches run at the warm clock);
# 2) PMC FETCH_SIZE pass; 3) PMC WRITE_SIZE pass -- separate runs.
set -o pipefail
tag=${1:-r01}; cfg=${2:-c4}; label=${3:-$cfg}
shift 3 2>/dev/null || shift $#
extra="$*"
export TMPDIR=/tmp
out=gpurun_out/prof_${tag}_${label}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 bench.py --profile --config $cfg --steps 30 $extra > $out/bench_trace.json 2> $out/trace.err || { tail -20 $out/trace.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- \
  python3 bench.py --profile --config $cfg --steps 3 --warmup 1 $extra > $out/bench_fetch.json 2> $out/fetch.err || { tail -20 $out/fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- \
  python3 bench.py --profile --config $cfg --steps 3 --warmup 1 $extra > $out/bench_write.json 2> $out/write.err || { tail -20 $out/write.err; exit 1; }
find $out -name "*.csv" | head -20
