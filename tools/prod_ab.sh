# Alternating-process warm A/B of the production-shape fused step (tools/prod_ab.py):
#   LIBS="ref srsrc ref:17" ROUNDS=3 bash tools/prod_ab.sh > out.jsonl
set -o pipefail
for r in $(seq ${ROUNDS:-3}); do
  for arm in ${LIBS:-ref srsrc}; do  # an arm: <lib>[:<digest variant>]
    lib=${arm%%:*}; v=""; [ "$arm" != "$lib" ] && v=${arm#*:}
    MDE_AB_VARIANT=$v MDE_LIBRARY=tools/abx/libmde_$lib.so timeout -k 10 120 python tools/prod_ab.py $lib 3 40 || exit 1
  done
done
