#!/bin/bash
# r03l: HBM traffic (FETCH_SIZE and WRITE_SIZE, one counter per pass) of the digest kernel alone and
# of the fused step on the B = 1,000 shapes: c4k (layout A, 1 KiB values), c4bk (layout B), ts8k
# (8-byte values, rec8). Run from the repo root on the GPU box:  bash tools/r03l_traffic.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03l; rm -rf gpurun_out/r03l/*
for what in digestonly:c4k fusedonly:c4k fusedonly:c4bk digestonly:ts8k fusedonly:ts8k; do
  tag=${what//:/_}
  for c in FETCH_SIZE WRITE_SIZE; do
    out=gpurun_out/r03l/${tag}_$c
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $out -o run -- python3 tools/microbench.py $what:3 > $out.log 2>&1 || { tail -5 $out.log; exit 1; }
  done
  grep -h "_us" gpurun_out/r03l/${tag}_FETCH_SIZE.log | tail -1
done
