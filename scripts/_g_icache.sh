#!/usr/bin/env bash
# instruction-cache counters of the render launches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ic
timeout -s KILL 60 rocprofv3 -L > gpurun_out/ic/avail.txt 2>&1
grep -iE "ICACHE|IFETCH|SQC_|INST_LEVEL|WAIT_INST|IFETCH" gpurun_out/ic/avail.txt | head -80 > gpurun_out/ic/avail_grep.txt
cat gpurun_out/ic/avail_grep.txt | cut -c1-200
TAG=ic/run BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --corrected-steps 0" \
PMC_SETS="SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU
SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" bash scripts/pmc_round.sh || exit $?
python3 scripts/pmc_dispatch.py gpurun_out/ic/run > gpurun_out/ic/dispatch.txt || exit $?
cat gpurun_out/ic/dispatch.txt
echo "=== done"
