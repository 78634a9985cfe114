# The GPU session launcher (run on the GPU box from the repo root). One tag, any of these steps,
# in order; each step runs under its own time limit and the script stops at the first failure.
#   TAG=r04a bash tools/gpu_round.sh tests smoke bench batch prof
# Steps:
#   tests   -m gpu parity suite            -> gpurun_out/$TAG/pytest_gpu.log
#   smoke   __graft_entry__.smoke()        -> smoke.log
#   bench   default bench line (N=1)       -> bench_default.json
#   batch   tests/cpp/batch_bench, 3 runs  -> batch_bench_r{1,2,3}.jsonl
#   group1  bench.py --engine group --gpus 1 (the N-GPU path as a 1-GPU group, RCCL) -> bench_group1.json
#   prod    bench.py --config prod line    -> bench_prod.json
#   prof    rocprofv3 trace + FETCH/WRITE PMC of the default bench (tools/profile.sh)
#   sq      SQ counters of the default bench workload (one --pmc pass)
#   service resident build service: server_test (1 / 10 / 8 callers, 100 and 2 ms lifetimes) and
#           the service + shim-replay pytest                         -> st{1,2,3}.json, service_pytest.log
#   callbench  batch_bench at B = 64 / 1,000 x 1 / 10 / 100 callers  -> bb.jsonl (+ summary)
#   stress  resident service under 4-64 callers, 1-100 ms lifetimes -> stress{1..5}.json
#   teardown  tools/stream_teardown phases a (minimal) and b (the service's sequence), once each
#           -> teardown_{a,b}.txt (run it last: a hang ends the call)
#   stepprobe fused-step per-wave timeline at the production shape (tools/step_probe.py, probe
#           library tools/ab/libmde_$PROBE_LIB.so, default stamps)        -> step_probe.jsonl
#   groupc  the multi-GPU path from plain C (tests/cpp/group_cabi.c; GROUPC_ARGS) -> group_cabi.json
#   groupbench bench.py --engine group at 1 GPU (RCCL) and 8 members on GPU 0 (--rehearse), C4 and C5
#           -> bench_group_{1,8}_{c4,c5}.json
#   serviceab bulk pipelined builds with no service / an idle one / one serving 10 callers
#           (tools/service_ab.py, C4 and PROD)                        -> service_ab_{c4,prod}.jsonl
#   cumask1   the service with MDE_SERVER_CUMASK=1 (its CU-masked stream destroyed with it): server_test
#           twice and tests/test_server.py once                        -> cumask1_*.txt / .log
#   testsall  -m gpu parity suite without -x (every failure listed)  -> pytest_gpu_all.log
#   callers the service at 10 / 100 callers with its wait totals (MDE_SERVER_DEBUG), user / system
#           CPU seconds and the cgroup's cpu.stat; SLOTS="16 32" sweeps the slot count -> callers.txt
# Extra bench flags: BENCH_ARGS="...".
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r04}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for s in "$@"; do
  case $s in
    tests)
      step tests
      timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
      tail -3 $O/pytest_gpu.log ;;
    testsall)
      step testsall
      timeout -k 10 1100 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread \
        > $O/pytest_gpu_all.log 2>&1 || { grep -E "FAILED|ERROR|Timeout" $O/pytest_gpu_all.log | head -40; tail -5 $O/pytest_gpu_all.log; exit 1; }
      tail -3 $O/pytest_gpu_all.log ;;
    topprobe)
      step topprobe  # A/B: the production-shape fused step with and without the wide trees' top levels
      for rep in 1 2 3; do
        for lib in mydatastore_amd/libmde.so tools/ab/libmde_${PROBE_LIB:-top64}.so; do
          MDE_LIBRARY=$lib timeout -k 10 180 python tools/top_probe.py $(basename $lib) 2 >> $O/top_probe.jsonl 2>> $O/top_probe.err \
            || { tail -20 $O/top_probe.err; exit 1; }
        done
      done
      cat $O/top_probe.jsonl ;;
    stepprobe)
      step stepprobe
      MDE_LIBRARY=tools/ab/libmde_${PROBE_LIB:-stamps}.so timeout -k 10 180 python tools/step_probe.py ${PROBE_ARGS:-} \
        > $O/step_probe.jsonl 2> $O/step_probe.err || { tail -20 $O/step_probe.err; exit 1; }
      cat $O/step_probe.jsonl ;;
    groupc)
      step groupc
      timeout -k 10 300 ./tests/cpp/build/group_cabi ${GROUPC_ARGS:-} > $O/group_cabi.json 2> $O/group_cabi.err || { tail -20 $O/group_cabi.err; exit 1; }
      cat $O/group_cabi.json ;;
    groupbench)
      step groupbench
      for spec in "1 c4" "1 c5" "8 c4" "8 c5"; do
        set -- $spec
        rh=""; [ $1 -gt 1 ] && rh="--rehearse"
        timeout -k 10 300 python bench.py --engine group --gpus $1 --config $2 $rh ${BENCH_ARGS:-} \
          > $O/bench_group_$1_$2.json 2> $O/bench_group_$1_$2.err || { tail -20 $O/bench_group_$1_$2.err; exit 1; }
        cat $O/bench_group_$1_$2.json
      done ;;
    serviceab)
      step serviceab
      for shp in c4 prod; do
        timeout -k 10 240 python tools/service_ab.py $shp 3 10 > $O/service_ab_$shp.jsonl 2> $O/service_ab_$shp.err || { tail -20 $O/service_ab_$shp.err; exit 1; }
        cat $O/service_ab_$shp.jsonl
      done ;;
    cumask1)
      step cumask1  # the resident service destroying its CU-masked stream with itself (MDE_SERVER_CUMASK=1)
      export MDE_SERVER_CUMASK=1 MDE_SERVER_DEBUG=1 MDE_TEARDOWN_TRACE=1
      for v in ${CUMASK_VARIANTS:-plain}; do
        f=$O/cumask1_$v.txt
        if [ $v = early ]; then export SERVER_TEST_EARLY_CTX=1; else unset SERVER_TEST_EARLY_CTX; fi
        timeout -k 10 90 tests/cpp/build/server_test 1 14 100 > $f 2>&1
        rc=$?; echo "exit status $rc" >> $f; cat $f
        [ $rc -eq 0 ] || exit 1
      done
      unset MDE_SERVER_DEBUG MDE_TEARDOWN_TRACE SERVER_TEST_EARLY_CTX
      if [ -n "${CUMASK_PYTEST:-}" ]; then
        timeout -k 10 400 python -u -m pytest tests/test_server.py tests/test_integration.py -m gpu -v -p no:cacheprovider \
          --timeout 120 --timeout-method thread > $O/cumask1_pytest.log 2>&1 || { tail -30 $O/cumask1_pytest.log; exit 1; }
        tail -3 $O/cumask1_pytest.log
      fi
      unset MDE_SERVER_CUMASK ;;
    teardown)
      step teardown
      for ph in ${TEARDOWN_PHASES:-a b}; do
        timeout -k 10 60 tools/stream_teardown $ph > $O/teardown_$ph.txt 2>&1
        rc=$?
        echo "exit status $rc" >> $O/teardown_$ph.txt
        cat $O/teardown_$ph.txt
        [ $rc -eq 0 ] || exit 1
      done ;;
    smoke)
      step smoke
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      cat $O/smoke.log ;;
    bench)
      step bench
      timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
      cat $O/bench_default.json ;;
    prod)
      step prod
      timeout -k 10 300 python bench.py --config prod ${BENCH_ARGS:-} > $O/bench_prod.json 2> $O/bench_prod.err || { tail -20 $O/bench_prod.err; exit 1; }
      cat $O/bench_prod.json ;;
    batch)
      step batch
      for rep in 1 2 3; do
        timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > $O/batch_bench_r$rep.jsonl 2> $O/batch_bench_r$rep.err || { tail -20 $O/batch_bench_r$rep.err; exit 1; }
        tail -1 $O/batch_bench_r$rep.jsonl
      done ;;
    group1)
      step group1
      timeout -k 10 300 python bench.py --engine group --gpus 1 ${BENCH_ARGS:-} > $O/bench_group1.json 2> $O/bench_group1.err || { tail -20 $O/bench_group1.err; exit 1; }
      cat $O/bench_group1.json ;;
    prof)
      step prof
      bash tools/profile.sh $TAG c4 c4 || exit 1 ;;
    sq)
      step sq
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
        --output-format csv -d $O/sq -o run -- python3 bench.py --profile ${BENCH_ARGS:-} --steps 3 --warmup 1 \
        > $O/sq.json 2> $O/sq.err || { tail -20 $O/sq.err; exit 1; } ;;
    service)
      step service
      i=0
      for a in "1 8 100" "10 40 100" "8 30 2"; do
        i=$((i+1))
        timeout -k 10 120 tests/cpp/build/server_test $a > $O/st$i.json 2> $O/st$i.err || { tail -5 $O/st$i.err; exit 1; }
        cat $O/st$i.json
      done
      timeout -k 10 300 python -u -m pytest tests/test_server.py tests/test_integration.py -m gpu -x -v -p no:cacheprovider \
        --timeout 120 --timeout-method thread > $O/service_pytest.log 2>&1 || { tail -30 $O/service_pytest.log; exit 1; }
      tail -3 $O/service_pytest.log ;;
    callbench)
      step callbench
      for B in 64 1000; do for P in 1 10 100; do
        timeout -k 10 150 tests/cpp/build/batch_bench 0.4 $B $P >> $O/bb.jsonl 2>> $O/bb.err || { tail $O/bb.err; exit 1; }
      done; done
      python tools/batch_summary.py $O/bb.jsonl ;;
    stress)
      step stress
      i=0
      for a in "32 40 1" "16 60 3" "64 10 1" "10 80 100" "4 200 1"; do
        i=$((i+1))
        timeout -k 10 150 tests/cpp/build/server_test $a > $O/stress$i.json 2> $O/stress$i.err || { tail -5 $O/stress$i.err; exit 1; }
        cat $O/stress$i.json
      done ;;
    callers)
      step callers
      TIMEFORMAT="time user %U sys %S wall %R"
      for sl in ${SLOTS:-16}; do
        for a in "64 10 server_hosttree" "64 100 server_hosttree" "64 100 verify_server" "1000 100 server_levels"; do
          echo "== $a slots $sl" >> $O/callers.txt
          cat /sys/fs/cgroup/cpu.stat >> $O/callers.txt 2>/dev/null || true
          { time MDE_SERVER_SLOTS=$sl MDE_SERVER_DEBUG=1 timeout -k 10 90 tests/cpp/build/batch_bench 0.4 $a \
              >> $O/callers.txt 2>&1 ; } 2>> $O/callers.txt || { tail $O/callers.txt; exit 1; }
        done
      done
      grep -E "^==|calls_per_s|for done|^time" $O/callers.txt | cut -c1-200 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
