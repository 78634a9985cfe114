set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04l}; mkdir -p $O
echo "== server_test 1x8"; timeout -k 10 60 tests/cpp/build/server_test 1 8 100 > $O/st1.json 2> $O/st1.err; rc=$?; cat $O/st1.json; tail -5 $O/st1.err; [ $rc -eq 0 ] || exit $rc
echo "== server_test 10x40"; timeout -k 10 90 tests/cpp/build/server_test 10 40 100 > $O/st2.json 2> $O/st2.err; rc=$?; cat $O/st2.json; tail -5 $O/st2.err; [ $rc -eq 0 ] || exit $rc
echo "== server_test 8x30 lifetime 2ms"; timeout -k 10 90 tests/cpp/build/server_test 8 30 2 > $O/st3.json 2> $O/st3.err; rc=$?; cat $O/st3.json; tail -5 $O/st3.err; [ $rc -eq 0 ] || exit $rc
echo "== batch_bench B=64/1000 x 1/10 callers"
for B in 64 1000; do for P in 1 10 100; do
  timeout -k 10 120 tests/cpp/build/batch_bench 0.4 $B $P >> $O/bb.jsonl 2>> $O/bb.err || { tail $O/bb.err; exit 1; }
done; done
python tools/batch_summary.py $O/bb.jsonl
echo "== pytest server + shim replay"; timeout -k 10 300 python -u -m pytest tests/test_server.py tests/test_integration.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -12 $O/pytest.log; exit $rc
