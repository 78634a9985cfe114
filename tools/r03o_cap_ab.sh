#!/bin/bash
# r03o: resident digest workgroups per CU (cap 2 = default, 3, 4) for the window / rec8 kernels
# at the reference's default B = 1,000: c4k (1 KiB values), ts8k (8-byte values); c4/8 as the
# shard-size check. Standalone digest and fused builds, one process, interleaved settings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/microbench.py pieces:d,d@3,d@4:c4k,ts8k,c4k/8 > gpurun_out/r03o_cap.jsonl 2> gpurun_out/r03o.err || { tail gpurun_out/r03o.err; exit 1; }
