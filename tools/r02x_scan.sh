# Prefix-scan path of the window kernel (steps with >= 2 bucket starts): pipeline parity tests,
# then the automatic choice vs round 1's kernel on production-sized values.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pipeline.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02x_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02x_pytest.log; [ $rc = 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r02x_pytest.log | head -60; exit 1; }
timeout -k 10 600 python -u tools/microbench.py pieces:x,d:ts8,ts8k,v64k,c4k,c4 > gpurun_out/r02x_scan.jsonl 2> gpurun_out/r02x.err || { tail gpurun_out/r02x.err; exit 1; }
cut -c1-230 gpurun_out/r02x_scan.jsonl
