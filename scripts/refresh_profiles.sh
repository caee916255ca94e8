#!/usr/bin/env bash
# Round profiles of the current build: bench line (with the CPU baseline), rocprofv3 kernel
# stats of the same command, PMC passes -> pmc_render.json (stamped with the timed kernel's code hash),
# then the bench line again reading that summary. Output under gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-final}
STEPS="bench prof" TAG=$T bash scripts/gpu_round.sh || exit $?
TAG=${T}_pmc bash scripts/pmc_round.sh || exit $?
timeout -k 10 300 python bench.py --pmc gpurun_out/${T}_pmc/pmc_render.json > gpurun_out/$T/bench_pmc.json 2> gpurun_out/$T/bench_pmc.err || exit $?
tail -1 gpurun_out/$T/bench_pmc.json
echo "=== done"
