#!/bin/bash
# r03f: SQ counters (two passes of <= 8 SQ counters each) of the fused step kernel on layout B at
# B = 1,000 vs B = 64 and of the 8-byte-record digest (item 5); run from the
# repo root on the GPU box:  bash tools/r03f_pmc.sh fusedonly:c4bk fusedonly:c4b digestonly:ts8k ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f; rm -rf gpurun_out/r03f/*
for what in "$@"; do
  tag=${what//:/_}
  out=gpurun_out/r03f/$tag
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
    --output-format csv -d $out/a -o run -- python3 tools/microbench.py $what:3 > $out.a.log 2>&1 || { tail -5 $out.a.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d $out/b -o run -- python3 tools/microbench.py $what:3 > $out.b.log 2>&1 || { tail -5 $out.b.log; exit 1; }
  grep -h "_us" $out.a.log | tail -1
done
