#!/usr/bin/env bash
# PMC passes (kernel-trace only, no sys/runtime trace) on a short bench, one counter set per pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline}
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "=== pass $i: $line"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $line --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; fi
  case $rc in 124|134|137|139) echo "stopping (rc=$rc)"; exit $rc ;; esac
done <<< "${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT
FETCH_SIZE
WRITE_SIZE}"
echo "=== done"
