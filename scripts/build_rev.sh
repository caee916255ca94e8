#!/usr/bin/env bash
# Build the product library of git revision <rev> into scripts/_abl/<name>/ (A/B against the
# working tree; rev WT = the working tree itself):   scripts/build_rev.sh <name> <rev> [-DFLAG ...]
set -eu
name=$1; rev=$2; shift 2
repo="$(cd "$(dirname "$0")/.." && pwd)"
src=$(mktemp -d)
for f in raytracinginoneweekend_amd/csrc/rt_kernel.hip raytracinginoneweekend_amd/csrc/rt_host.cpp \
         raytracinginoneweekend_amd/csrc/rt_device.h include/rt_api.h; do
  mkdir -p "$src/$(dirname $f)"
  if [ "$rev" = WT ]; then cp "$repo/$f" "$src/$f"; else git -C "$repo" show "$rev:$f" > "$src/$f"; fi
done
out=$repo/scripts/_abl/$name
mkdir -p $out
FLAGS="-std=c++17 -O3 -fno-slp-vectorize --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -Wall"
cd "$src/raytracinginoneweekend_amd/csrc"
/opt/rocm/bin/hipcc $FLAGS "$@" -c rt_kernel.hip -o $out/rt_kernel.o &
/opt/rocm/bin/hipcc $FLAGS "$@" -x hip -c rt_host.cpp -o $out/rt_host.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/librt_mi355x.so $out/rt_kernel.o $out/rt_host.o -Wl,--no-undefined
rm -rf "$src"
echo "built $out/librt_mi355x.so ($rev)"
