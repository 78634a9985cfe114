# Window variants (13/14: register window over bucket starts, true double buffer, batched
# window atomics) vs the defaults (11/12): parity tests, then same-process A/B at B = 64, B = 1000
# (the reference's default PartitionBuckets) and C3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_pipeline.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02u_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02u_pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 700 python -u tools/microbench.py pieces:d,v13d,x,v13x:c4,c4k,c4/8,c4k/8,c3 > gpurun_out/r02u_window.jsonl 2> gpurun_out/r02u.err || { tail gpurun_out/r02u.err; exit 1; }
cut -c1-230 gpurun_out/r02u_window.jsonl
