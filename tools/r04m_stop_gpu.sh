# resident service: stream kind vs teardown and vs the batcher's streams (diagnostics)
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
echo "== batch_bench with the service on a plain stream"
for B in 64 1000; do timeout -k 5 120 tests/cpp/build/batch_bench 0.4 $B 10 >> $O/bb.jsonl 2>> $O/bb.err || { tail $O/bb.err; exit 1; }; done
python tools/batch_summary.py $O/bb.jsonl
echo "== server_test 10x40, plain stream"; timeout -k 5 90 tests/cpp/build/server_test 10 40 100 > $O/st10.json 2> $O/st10.err; rc=$?; cat $O/st10.json; tail -3 $O/st10.err; [ $rc -eq 0 ] || exit $rc
echo "== server_test 1x8, CU-masked stream kept"; MDE_SERVER_DEBUG=1 MDE_SERVER_CUMASK=2 timeout -k 5 40 tests/cpp/build/server_test 1 8 100 > $O/st2.json 2> $O/st2.err; rc=$?; cat $O/st2.json; tail -8 $O/st2.err; exit $rc
