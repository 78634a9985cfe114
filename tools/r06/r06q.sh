# Host CPU the group engine burns (the enqueue threads' spin): the bench line's
# host_timing.host_cpu_cores at N = 1 and for an 8-member group on one GPU, with the enqueue
# threads (default) and without (MDE_GROUP_THREADS=0, every device call from the caller's thread).
set -o pipefail
cd $GRAFT_REPO_ROOT
b="python -u bench.py --steps 40 --no-cpu-baseline --no-e2e --no-production-shape"
timeout -k 10 200 $b > gpurun_out/r06q_n1.json 2> gpurun_out/r06q_n1.err &&
timeout -k 10 200 $b --gpus 8 --rehearse --no-gather-per-build > gpurun_out/r06q_g8_threads.json 2> gpurun_out/r06q_g8_threads.err &&
MDE_GROUP_THREADS=0 timeout -k 10 200 $b --gpus 8 --rehearse --no-gather-per-build > gpurun_out/r06q_g8_nothreads.json 2> gpurun_out/r06q_g8_nothreads.err &&
timeout -k 10 200 $b --config c5 --gpus 8 --rehearse --no-gather-per-build > gpurun_out/r06q_c5g8_threads.json 2> gpurun_out/r06q_c5g8_threads.err &&
MDE_GROUP_THREADS=0 timeout -k 10 200 $b --config c5 --gpus 8 --rehearse --no-gather-per-build > gpurun_out/r06q_c5g8_nothreads.json 2> gpurun_out/r06q_c5g8_nothreads.err
