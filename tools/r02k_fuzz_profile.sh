# r02k: long decode/verify fuzz (incl. deep unknown groups, caps 64 and 512), then rocprofv3
# profiles of the default bench (C4, automatic digest pieces) and of C3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/fuzz_long.py 2 20000 300 > gpurun_out/r02k_fuzz_long.jsonl 2> gpurun_out/r02k_fuzz.err || { tail -20 gpurun_out/r02k_fuzz.err; exit 1; }
cat gpurun_out/r02k_fuzz_long.jsonl | cut -c1-200
bash tools/profile.sh r02k c4 c4 || exit 1
bash tools/profile.sh r02k c3 c3 || exit 1
