# Fused build step at B > 128: the pair-shape trees (`base`: two partitions per workgroup, top
# levels of both in one wave, at >= 512 partitions; `pair0`: at any partition count) vs the
# previous library's two-wave trees (`head`), and `top` = head with every tree stopped at its first
# level of <= 64 nodes (wrong roots; tools/build_probe_lib.sh top -DMDE_PROBE_TREE_TOP): the most
# that cheaper top levels could win. Parity of the pair shape first. Alternating processes.
# (At the time of the run `base` used the pair shape in the fused step too; the product keeps it
# only in the standalone tree kernel. The MDE_PROBE_TREE_TOP switch was removed after the run.)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pair_pytest.log 2>&1 || { tail -30 gpurun_out/pair_pytest.log; exit 1; }
tail -2 gpurun_out/pair_pytest.log
for rep in 1 2; do for lib in base pair0 head top; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 150 python tools/microbench.py pieces:d:ts8k,v64k,c4k,c4k/8 > gpurun_out/treetop.log 2>&1 || { tail gpurun_out/treetop.log; exit 1; }
  grep '"shape"' gpurun_out/treetop.log | sed "s/^{/{\"rep\": $rep, \"lib\": \"$lib\", /"
done; done
