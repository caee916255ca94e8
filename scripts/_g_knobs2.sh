#!/usr/bin/env bash
# scene/culling knobs re-swept on the current kernel (config 3 frame stream)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=knobs2 SETS1="-;RT_CLUSTER_SIZE=12;RT_CLUSTER_SIZE=20;RT_CLUSTER_SIZE=24;RT_TRANSPOSE_MAX=8;RT_TRANSPOSE_MAX=12" R1=2 bash scripts/_g_ab.sh || exit 1
echo "=== done"
