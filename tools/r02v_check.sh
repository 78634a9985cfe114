# Full GPU suite + smoke + default bench, then the automatic variant choice vs round 1's kernel.
set -o pipefail
bash tools/gpu_tests_bench.sh || exit 1
timeout -k 10 700 python -u tools/microbench.py pieces:x,d:c4,c4k,c4k/8,c3 > gpurun_out/r02v_auto.jsonl 2> gpurun_out/r02v.err || { tail gpurun_out/r02v.err; exit 1; }
cut -c1-230 gpurun_out/r02v_auto.jsonl
