#!/usr/bin/env bash
# generic A/B: SETS1 on config 3, SETS8 on the 8-way share
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-ab}
[ -n "${SETS1:-}" ] && { TAG=$T/c3 SETS="$SETS1" ROUNDS=${R1:-2} bash scripts/ab_env3.sh || exit 1; }
[ -n "${SETS8:-}" ] && { TAG=$T/s8 SETS="$SETS8" ROUNDS=${R8:-2} ARGS="--rehearse-world 8" bash scripts/ab_env3.sh || exit 1; }
[ -n "${SETS4:-}" ] && { TAG=$T/s4 SETS="$SETS4" ROUNDS=${R4:-2} ARGS="--rehearse-world 4" bash scripts/ab_env3.sh || exit 1; }
echo "=== all done"
