# Instruction-cache counters of the production shape's fused step vs the digest alone (one --pmc
# pass each; run from the repo root on the GPU box):  bash tools/icache_pmc.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-icache}; mkdir -p $O
for what in fusedonly:ts8k digestonly:ts8k; do
  tag=${what//:/_}
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
    --output-format csv -d $O/$tag -o run -- python3 tools/microbench.py $what:3 > $O/$tag.log 2>&1 || { tail -8 $O/$tag.log; exit 1; }
  grep -h "_us" $O/$tag.log | tail -1
done
