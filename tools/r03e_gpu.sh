#!/bin/bash
# r03e: record-space 8-byte digest (variants 15/16): full GPU suite, then A/B against the window
# kernel (variant 13) on 8-byte shapes -- standalone digest and fused builds, interleaved.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03e_pytest.log 2>&1 &&
timeout -k 10 300 python tools/microbench.py pieces:d,v13d:ts8k,ts8,v64k,c4k > gpurun_out/r03e_ab.jsonl 2> gpurun_out/r03e_ab.err
