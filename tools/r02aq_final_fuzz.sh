# Round-2 final tree: GPU suite, then the build fuzz (4 seeds x 200 cases vs the C oracle) and the
# long decode/verify fuzz (caps 64 and 512, deep unknown groups) on the shipped library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for seed in 5 6 7 8; do
  MDE_FUZZ_SEED=$seed MDE_FUZZ_CASES=200 timeout -k 10 400 python -u -m pytest tests/test_fuzz.py -x -q -p no:cacheprovider --timeout 380 --timeout-method thread > gpurun_out/r02aq_fuzz_$seed.log 2>&1 || { tail -30 gpurun_out/r02aq_fuzz_$seed.log; exit 1; }
  echo "seed $seed: $(tail -1 gpurun_out/r02aq_fuzz_$seed.log)"
done
timeout -k 10 600 python -u tools/fuzz_long.py 3 20000 300 > gpurun_out/r02aq_fuzz_long.jsonl 2> gpurun_out/r02aq_fuzz_long.err || { tail -20 gpurun_out/r02aq_fuzz_long.err; exit 1; }
cut -c1-300 gpurun_out/r02aq_fuzz_long.jsonl
