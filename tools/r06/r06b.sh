set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pipeline.py -k "rec8_ragged or every_digest_variant_matches_golden" > gpurun_out/r06b_pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/rec8_variant_check.py 19 20 > gpurun_out/r06b_check.jsonl 2>&1 &&
for r in 1 2 3; do
  for v in 15 19; do
    MDE_AB_VARIANT=$v timeout -k 10 120 python tools/prod_ab.py lib 3 40 >> gpurun_out/r06b_ab.jsonl 2>&1 || exit 1
  done
done
