#!/usr/bin/env bash
# Build an A/B variant of the product library with extra defines into scripts/_abl/<name>/.
#   scripts/build_variant.sh <name> -DFLAG ...   ->  RT_LIB_PATH=scripts/_abl/<name>/librt_mi355x.so
set -eu
name=$1; shift
cd "$(dirname "$0")/../raytracinginoneweekend_amd/csrc"
out=../../scripts/_abl/$name
mkdir -p $out
FLAGS="-std=c++17 -O3 -fno-slp-vectorize --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -Wall"
/opt/rocm/bin/hipcc $FLAGS "$@" -c rt_kernel.hip -o $out/rt_kernel.o
/opt/rocm/bin/hipcc $FLAGS "$@" -x hip -c rt_host.cpp -o $out/rt_host.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/librt_mi355x.so $out/rt_kernel.o $out/rt_host.o -Wl,--no-undefined
echo "built $out/librt_mi355x.so"
