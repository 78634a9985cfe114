set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for lib in base noatomic noreduce none; do
  if [ $lib = base ]; then unset MDE_LIBRARY; else export MDE_LIBRARY=tools/ab/libmde_$lib.so; fi
  timeout -k 10 200 python -u tools/microbench.py pieces:v13x:c4k > gpurun_out/r02t_$lib.jsonl 2> gpurun_out/r02t.err || { tail gpurun_out/r02t.err; exit 1; }
  sed "s/^/$lib $rep /" gpurun_out/r02t_$lib.jsonl | cut -c1-200
done; done
