#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-pmc2} BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --corrected-steps 0" bash scripts/pmc_round.sh || exit $?
python3 scripts/pmc_dispatch.py gpurun_out/${TAG:-pmc2} > gpurun_out/${TAG:-pmc2}/dispatch.txt || exit $?
cat gpurun_out/${TAG:-pmc2}/dispatch.txt
echo "=== done"
