# Register window over the bucket starts (digest variants 13/14) vs the round-1 default (11/12):
# parity tests, then same-process A/B at B = 64 and B = 1000 (the reference's default
# PartitionBuckets), N=1 shape and the N=8 strong shard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_pipeline.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02s_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02s_pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u tools/microbench.py pieces:d,v13d,x,v13x:c4,c4k,c4/8,c4k/8 > gpurun_out/r02s_window.jsonl 2> gpurun_out/r02s.err || { tail gpurun_out/r02s.err; exit 1; }
cat gpurun_out/r02s_window.jsonl
