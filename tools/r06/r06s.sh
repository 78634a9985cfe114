# Which leg before bench's production_shape slows its digest-alone reading (r06r: 156 us in the
# full line, 141 in tools/idle_probe.py on the same box): the line with the CPU baseline and/or the
# end-to-end leg switched off, then both on.
set -o pipefail
cd $GRAFT_REPO_ROOT
b="python -u bench.py --steps 5"
timeout -k 10 300 $b --no-cpu-baseline --no-e2e > gpurun_out/r06s_none.json 2> gpurun_out/r06s_none.err &&
timeout -k 10 300 $b --no-cpu-baseline > gpurun_out/r06s_e2e.json 2> gpurun_out/r06s_e2e.err &&
timeout -k 10 300 $b --no-e2e > gpurun_out/r06s_cpu.json 2> gpurun_out/r06s_cpu.err &&
timeout -k 10 300 $b > gpurun_out/r06s_both.json 2> gpurun_out/r06s_both.err
