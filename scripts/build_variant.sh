#!/usr/bin/env bash
# Build librt_mi355x.so with extra compile-time definitions into scripts/_abl/<name>/ (A/B builds,
# loaded through RT_LIB_PATH; not tracked):  bash scripts/build_variant.sh <name> -DRT_X=1 ...
set -eu
cd "$(dirname "$0")/../raytracinginoneweekend_amd/csrc"
name=$1; shift
mkdir -p ../../scripts/_abl/$name
make -s OBJ=_obj_abl/$name OUT=../../scripts/_abl/$name/librt_mi355x.so \
     FLAGS="-std=c++17 -O3 -fno-slp-vectorize --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -Wall $*"
echo "built scripts/_abl/$name/librt_mi355x.so ($*)"
