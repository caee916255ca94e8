#!/usr/bin/env bash
# shared rejection: plain attempts before sharing 2 (product build) / 3 / 1 vs head
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=$PWD/scripts/_abl
TAG=share2/ab SETS1="-;RT_LIB_PATH=$L/head/librt_mi355x.so;RT_LIB_PATH=$L/p3/librt_mi355x.so;RT_LIB_PATH=$L/p1/librt_mi355x.so" R1=3 bash scripts/_g_ab.sh || exit 1
echo "=== done"
