#!/usr/bin/env bash
# Config-3 8-way row share (rank 0 of 8, rehearsed on one GPU): per-dispatch PMC issue counts
# and the instrumented kernel's drain statistics, next to the full frame's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r3diag}
mkdir -p "$O"
export TMPDIR=/tmp
for n in 8 1; do
  A="--no-cpu-baseline --corrected-steps 0 --steps 6 --warmup 2"
  [ $n -gt 1 ] && A="$A --rehearse-world $n"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc$n" -o run -- python3 bench.py $A > "$O/pmc$n.log" 2>&1 || exit $?
done
for n in 8 1; do
  timeout -k 10 120 python scripts/timeline_c3.py --rehearse-world $n > "$O/stats_tl$n.json" 2>&1 || exit $?
  tail -30 "$O/stats_tl$n.json"
done
for e in "" "RT_DEEP_MIN_ITEMS=0" "RT_GRID_WG_PER_CU=1" "RT_GRID_WG_PER_CU=3" "RT_PIPELINE=3" ; do
  env $e timeout -k 10 120 python bench.py --rehearse-world 8 --no-cpu-baseline --corrected-steps 0 --steps 40 --warmup 3 > "$O/ab.json" 2>/dev/null || exit $?
  tail -1 "$O/ab.json" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('[$e]', r['ms_per_step'], r['frame_device_ms'])"
done
echo "=== done"
