#!/usr/bin/env bash
# The round's evidence on one MI355X, in the order the judged files depend on each other:
# smoke and the GPU tests, the PMC passes (pmc_render.json stamped with the timed kernels' code
# hash), the bench line reading that summary, rocprofv3 kernel stats of the same command, then the
# N = 1/2/4/8 row-share rehearsals. Every step has its own time limit; the first failure ends it.
# Outputs under gpurun_out/$TAG*; copy into profiles/ what is judged (DESIGN.md §6-§8 name them).
#   TAG=r05_final bash scripts/round_evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-evidence}
TAG=$T STEPS="smoke pytest" STRICT=1 bash scripts/gpu_round.sh || exit $?
TAG=${T}pmc bash scripts/pmc_round.sh || exit $?
cp gpurun_out/${T}pmc/pmc_render.json profiles/pmc_render_c3.json  # (this copy of the tree: the bench reads it)
TAG=$T STEPS="bench prof" STRICT=1 bash scripts/gpu_round.sh || exit $?
mkdir -p gpurun_out/${T}reh
for n in 1 2 4 8; do
  if [ $n = 1 ]; then a=""; else a="--rehearse-world $n --rehearse-gather"; fi
  timeout -k 10 300 python bench.py $a --no-cpu-baseline --corrected-steps 0 > gpurun_out/${T}reh/n$n.json 2> gpurun_out/${T}reh/n$n.err || exit $?
done
echo ALLDONE
