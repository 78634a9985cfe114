# Long build fuzz on the round-2 digest paths (automatic variant choice: window kernel, prefix-scan
# path, pieces; layout-B small records): 4 extra seeds x 200 cases vs the C oracle.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for seed in 1 2 3 4; do
  MDE_FUZZ_SEED=$seed MDE_FUZZ_CASES=200 timeout -k 10 400 python -u -m pytest tests/test_fuzz.py -x -q -p no:cacheprovider --timeout 380 --timeout-method thread > gpurun_out/r02ab_fuzz_$seed.log 2>&1 || { tail -30 gpurun_out/r02ab_fuzz_$seed.log; exit 1; }
  echo "seed $seed: $(tail -1 gpurun_out/r02ab_fuzz_$seed.log)"
done
