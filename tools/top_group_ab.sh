# The fused step's group pass over the trees' top levels: parity, then A/B of MDE_STEP_TOP_GROUP
# (0 = off, 4, 8) on the production shape and C4 at B = 1,000, alternating processes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-topab}; mkdir -p $O
MDE_STEP_TOP_GROUP=4 timeout -k 10 400 python -u -m pytest tests/test_step_top.py tests/test_pipeline.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for rep in 1 2; do for g in 0 4 8; do  # (default 0)
  MDE_STEP_TOP_GROUP=$g timeout -k 10 200 python bench.py --config prod --steps 40 --warmup 5 > $O/prod_g$g.r$rep.json 2> $O/prod_g$g.r$rep.err || { tail -5 $O/prod_g$g.r$rep.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$O/prod_g$g.r$rep.json'));ps=d['production_shape'];print('prod g=$g r$rep', d['ms_per_step'], ps['fused_us_per_build'], ps['equals_c_oracle_on_sample'], d['parity']['all_ranks_ok'])"
done; done
for g in 0 4; do
  MDE_STEP_TOP_GROUP=$g timeout -k 10 200 python bench.py --config c4k --steps 20 --warmup 3 > $O/c4k_g$g.json 2> $O/c4k_g$g.err || { tail -5 $O/c4k_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c4k_g$g.json'));print('c4k g=$g', d['ms_per_step'], d['parity']['all_ranks_ok'])"
done
