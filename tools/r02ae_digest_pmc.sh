# SQ counters of the default digest kernel alone, per workload shape (run on the GPU box from the
# repo root): instruction mix and wait cycles, to see what bounds the small-bucket paths.
#   bash tools/r02ae_digest_pmc.sh ts8k c4k c4
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ae
for shape in "$@"; do
  out=gpurun_out/r02ae/$shape
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
    --output-format csv -d $out/a -o run -- python3 tools/microbench.py digestonly:$shape:3 > $out.a.log 2>&1 || { tail -5 $out.a.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d $out/b -o run -- python3 tools/microbench.py digestonly:$shape:3 > $out.b.log 2>&1 || { tail -5 $out.b.log; exit 1; }
  grep digest_us $out.a.log
done
find gpurun_out/r02ae -name "*counter_collection.csv" | head
