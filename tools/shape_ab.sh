# Alternating-process warm A/B of one shape's fused step over probe libraries (tools/shape_probe.py):
#   SHAPE="10000000 1024 1024 1000" LIBS="ref tlast" ROUNDS=3 bash tools/shape_ab.sh > out.jsonl
set -o pipefail
for r in $(seq ${ROUNDS:-3}); do
  for lib in ${LIBS:-ref}; do
    MDE_LIBRARY=tools/ab/libmde_$lib.so timeout -k 10 150 python tools/shape_probe.py ${SHAPE:-10000000 1024 1024 1000} 2 \
      | sed "s/^{/{\"lib\": \"$lib\", /" || exit 1
  done
done
