# Build a probe copy of libmde.so with extra compile definitions (A/B only, never the product):
#   bash tools/build_probe_lib.sh <name> -DMDE_PROBE_X ...   ->  tools/ab/libmde_<name>.so
set -e
name=$1; shift
out=tools/ab/probe_$name
mkdir -p $out tools/ab
for src in mydatastore_amd/csrc/*.hip; do
  hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-function -Iinclude "$@" -x hip -c $src -o $out/$(basename $src .hip).o
done
hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Iinclude "$@" -c mydatastore_amd/csrc/mde_api.cpp -o $out/mde_api.o
hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Iinclude "$@" -c mydatastore_amd/csrc/batch.cpp -o $out/batch.o
hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Iinclude "$@" -c mydatastore_amd/csrc/group.cpp -o $out/group.o
hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Iinclude "$@" -c mydatastore_amd/csrc/server.cpp -o $out/server.o
hipcc -shared --offload-arch=gfx950 -pthread -o tools/ab/libmde_$name.so $out/*.o -ldl
rm -rf $out
echo tools/ab/libmde_$name.so
