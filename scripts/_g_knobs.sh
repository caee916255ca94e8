#!/usr/bin/env bash
# scheduling knobs re-swept on the current kernel (config 3 frame stream; 8-way share)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=knobs SETS1="-;RT_GRID_WG_PER_CU=3;RT_GRID_WG_PER_CU=5;RT_GRID_WG_PER_CU=7;RT_PIPELINE=5;RT_TAIL_PCT=4;RT_TAIL_PCT=16" R1=2 \
SETS8="-;RT_GRID_WG_PER_CU=1;RT_GRID_WG_PER_CU=3;RT_PIPELINE=5" R8=2 bash scripts/_g_ab.sh || exit 1
echo "=== done"
