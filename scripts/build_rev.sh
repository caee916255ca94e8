#!/usr/bin/env bash
# Build the product library of git revision <rev> into scripts/_abl/<name>/ (A/B against the
# working tree; rev WT = the working tree itself), with that revision's own Makefile:
#   scripts/build_rev.sh <name> <rev> [-DFLAG ...]
set -eu
name=$1; rev=$2; shift 2
repo="$(cd "$(dirname "$0")/.." && pwd)"
src=$(mktemp -d)
if [ "$rev" = WT ]; then
  cp -r "$repo/raytracinginoneweekend_amd" "$repo/include" "$src/"
  rm -rf "$src/raytracinginoneweekend_amd/csrc/_obj"*
else
  git -C "$repo" archive "$rev" raytracinginoneweekend_amd/csrc include | tar -x -C "$src"
fi
out=$repo/scripts/_abl/$name
mkdir -p "$out"
make -s -C "$src/raytracinginoneweekend_amd/csrc" OBJ="$src/_obj" OUT="$out/librt_mi355x.so" \
     FLAGS="-std=c++17 -O3 -fno-slp-vectorize --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -Wall $*"
rm -rf "$src"
echo "built scripts/_abl/$name/librt_mi355x.so ($rev $*)"
