#!/bin/bash
# r03t: batcher write-once outputs in pinned memory (MDE_DIRECT_OUT=1) vs D2H copies (=0),
# alternating processes, 3 repetitions of batch_bench.
set -o pipefail
mkdir -p gpurun_out/r03t; rm -rf gpurun_out/r03t/*
for rep in 1 2 3; do for d in 1 0; do
  MDE_DIRECT_OUT=$d timeout -k 10 300 tests/cpp/build/batch_bench 0.4 > gpurun_out/r03t/d${d}_$rep.jsonl 2>> gpurun_out/r03t/err || exit 1
done; done
