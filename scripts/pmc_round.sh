#!/usr/bin/env bash
# PMC passes (kernel-trace only, no sys/runtime trace) over a short bench.py run, one counter set
# per pass (each set within the per-block limits), then the JSON bench.py reads.
#   TAG=name BENCH_ARGS="..." bash scripts/pmc_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --corrected-steps 0 --no-dropin}
# (--no-dropin: the drop-in timing renders frames through another scene, which the PMC sums would
# count and frames_issued would not)
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "=== pass $i: $line"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $line --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<< "${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH
SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64
FETCH_SIZE
WRITE_SIZE}"
python3 scripts/pmc_json.py "$OUT" "$OUT/pmc_render.json" ${PMC_JSON_ARGS:-}
python3 scripts/pmc_summary.py "$OUT" "render_kernel" > "$OUT/pmc_render.txt"
python3 scripts/pmc_summary.py "$OUT" "accumulate_kernel" > "$OUT/pmc_accumulate.txt"
echo "=== done"
