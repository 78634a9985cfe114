#!/bin/bash
# r03w: rec8 with its range bounds in SGPRs (no buffer-load waterfall loops): rec8 parity tests,
# ts8k / ts8 timing, fused-step stamps (probe lib), SQ counters of the ts8k digest and fused step.
set -o pipefail
mkdir -p gpurun_out/r03w; rm -rf gpurun_out/r03w/*
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py -m gpu -q -k "rec8 or default_variant or tagged_equals or fused_step" --timeout 250 --timeout-method thread > gpurun_out/r03w/pytest.log 2>&1 || { tail -30 gpurun_out/r03w/pytest.log; exit 1; }
tail -1 gpurun_out/r03w/pytest.log
timeout -k 10 200 python tools/microbench.py pieces:d:ts8k,ts8,c4k > gpurun_out/r03w/ab.jsonl 2> gpurun_out/r03w/ab.err || exit 1
cat gpurun_out/r03w/ab.jsonl
MDE_LIBRARY=tools/ab/libmde_stamps.so timeout -k 10 120 python tools/microbench.py stamps:ts8k > gpurun_out/r03w/stamps.txt 2>> gpurun_out/r03w/ab.err || exit 1
MDE_LIBRARY=tools/ab/libmde_stamps.so timeout -k 10 120 python tools/microbench.py stamps:c4k >> gpurun_out/r03w/stamps.txt 2>> gpurun_out/r03w/ab.err || exit 1
cat gpurun_out/r03w/stamps.txt
bash tools/r03f_pmc.sh digestonly:ts8k fusedonly:ts8k > gpurun_out/r03w/pmc.log 2>&1
