# Build a probe copy of libmde.so (A/B and timelines only, never the product): the product sources
# copied to a scratch tree, the given patches applied (tools/probe_*.patch, e.g. the per-wave
# timeline stamps that tools/step_probe.py and placement_probe.py read), the given compile flags:
#   bash tools/build_probe_lib.sh <name> [x.patch ...] [-DFLAG ...]  ->  tools/abx/libmde_<name>.so
# The product sources carry no probe code; a patch that no longer applies
# fails the build here, not silently.
set -e
name=$1; shift
patches=(); flags=()
for a in "$@"; do case "$a" in *.patch) patches+=("$(realpath "$a")");; *) flags+=("$a");; esac; done
src=$(mktemp -d)
mkdir -p "$src/mydatastore_amd"
cp -r mydatastore_amd/csrc "$src/mydatastore_amd/csrc"
cp -r include "$src/include"
c=$src/mydatastore_amd/csrc
for p in "${patches[@]}"; do (cd "$c" && patch -p1 --no-backup-if-mismatch < "$p"); done
out=$src/obj; mkdir -p $out tools/abx
pids=()
for f in $c/*.hip; do
  hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-function -I$src/include "${flags[@]}" -x hip -c $f -o $out/$(basename $f .hip).o &
  pids+=($!)
done
for f in mde_api batch group server; do
  hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -I$src/include "${flags[@]}" -c $c/$f.cpp -o $out/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
hipcc -shared --offload-arch=gfx950 -pthread -o tools/abx/libmde_$name.so $out/*.o -ldl
rm -rf "$src"
echo tools/abx/libmde_$name.so
