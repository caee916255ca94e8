#!/usr/bin/env bash
# root-form hoist + ground block: parity subset, A/B against head (and the no-ground-block build), SALU PMC
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${T:-hoist}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1; rc=$?
tail -3 $O/pytest_parity.log
[ $rc -eq 0 ] || exit $rc
H=RT_LIB_PATH=$PWD/scripts/_abl/head/librt_mi355x.so
G=${G:-}
TAG=${T:-hoist}/ab SETS1="-;$H${G:+;$G}" R1=${R1:-3} SETS8="-;$H" R8=2 bash scripts/_g_ab.sh || exit 1
TAG=${T:-hoist}/pmc BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --corrected-steps 0" \
PMC_SETS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES" bash scripts/pmc_round.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 scripts/pmc_dispatch.py --timed gpurun_out/${T:-hoist}/pmc > $O/pmc.txt || exit 1
cat $O/pmc.txt
echo "=== done"
