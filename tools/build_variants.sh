#!/bin/bash
# Dev tool: build A/B variants of liblincheck.so with -D switches into
# gpurun-shipped build dirs: tools/variants/<name>/liblincheck.so
#   tools/build_variants.sh <name> [-DSWITCH=value ...]
# (then tools/ab_bench.sh benches every directory under tools/variants)
set -e
cd "$(dirname "$0")/../jepsen/etcd_amd/csrc"
name=$1; shift
out=../../../tools/variants/$name
mkdir -p $out/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c check_kernel.hip -o $out/obj/k.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c gap_tier.hip -o $out/obj/g.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c fx.hip -o $out/obj/f.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c cert.hip -o $out/obj/c.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC "$@" -x hip --offload-arch=gfx950 -DLC_BUILD_ID='"variant"' -c lincheck.cpp -o $out/obj/h.o
g++ -O3 -std=c++17 -fPIC -c synth.cpp -o $out/obj/s.o
g++ -O3 -std=c++17 -fPIC -c edn.cpp -o $out/obj/e.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/liblincheck.so $out/obj/*.o -lpthread -ldl
rm -rf $out/obj
