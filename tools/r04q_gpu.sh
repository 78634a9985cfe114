# resident service stress: many callers, 1 ms lifetime (relaunch races), repeated; Python tests
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
i=0
for args in "32 40 1" "16 60 3" "64 10 1" "10 80 100" "4 200 1"; do
  i=$((i+1)); echo "== server_test $args"
  timeout -k 10 150 tests/cpp/build/server_test $args > $O/st$i.json 2> $O/st$i.err || { tail -5 $O/st$i.err; exit 1; }
  cat $O/st$i.json
done
timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -10 $O/pytest.log; exit $rc
