# resident service wait policy at 10 / 100 callers + the round's rocprofv3 profile of the default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
echo "== service rows"
for B in 64 1000; do for P in 10 100; do for c in server server_hosttree verify_server; do
  timeout -k 5 60 tests/cpp/build/batch_bench 0.4 $B $P $c >> $O/bb.jsonl 2>> $O/bb.err || { tail $O/bb.err; exit 1; }
done; done; done
python tools/batch_summary.py $O/bb.jsonl
echo "== server_test 10x40"; timeout -k 10 90 tests/cpp/build/server_test 10 40 100 > $O/st2.json 2> $O/st2.err || { tail $O/st2.err; exit 1; }; cat $O/st2.json
echo "== prof"; bash tools/profile.sh r04p c4 c4 || exit 1
echo "== group1"; TAG=r04p bash tools/gpu_round.sh group1
