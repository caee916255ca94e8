#!/usr/bin/env bash
# instruction counts (VALU, SALU, branch) of the main launch per duplication-ablation build:
# each build runs one part of the loop twice, so build - head = that part's instructions
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dupsalu
for b in head ${BUILDS:-reject hit boxes2 ground members_t members_l refract}; do
  d=scripts/_abl/$b; [ "$b" != head ] && d=scripts/_abl/dup_$b
  echo "=== $b"
  RT_LIB_PATH=$PWD/$d/librt_mi355x.so TAG=dupsalu/$b BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --corrected-steps 0" \
  PMC_SETS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES" bash scripts/pmc_round.sh > gpurun_out/dupsalu/$b.log 2>&1 || { tail -5 gpurun_out/dupsalu/$b.log; exit 1; }
  python3 scripts/pmc_dispatch.py --timed gpurun_out/dupsalu/$b > gpurun_out/dupsalu/$b.txt || exit 1
  cat gpurun_out/dupsalu/$b.txt
done
echo "=== done"
