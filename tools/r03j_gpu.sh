#!/bin/bash
# r03j: GPU suite, default bench line, rocprofv3 trace + FETCH/WRITE PMC of the bench's C4 step,
# and SQ counters of the round-3 kernels (rec8 digest / fused step at ts8k, layout-B fused steps).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03j_pytest.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r03j_bench.json 2> gpurun_out/r03j_bench.err &&
bash tools/profile.sh r03j c4 c4 > gpurun_out/r03j_profile.log 2>&1 &&
bash tools/r03f_pmc.sh digestonly:ts8k fusedonly:ts8k fusedonly:c4bk fusedonly:c4b > gpurun_out/r03j_pmc.log 2>&1
