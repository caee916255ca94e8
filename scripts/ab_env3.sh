#!/usr/bin/env bash
# Interleaved A/B of environment settings on one bench workload: ROUNDS rounds, each running
# every setting of $SETS (';'-separated lists of VAR=value, "-" = defaults) once.
#   TAG=x SETS="-;RT_HOT_FIRST=0" ARGS="--rehearse-world 8" ROUNDS=3 bash scripts/ab_env3.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p "$O"
IFS=';' read -ra S <<< "${SETS:--}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in "${S[@]}"; do
    [ "$e" = "-" ] && ev="" || ev="$e"
    env $ev timeout -k 10 ${STEP_TIMEOUT:-200} python bench.py --no-cpu-baseline --corrected-steps ${CSTEPS:-0} ${ARGS:-} > "$O/ab.json" 2> "$O/ab.err" || { echo "FAILED [$e]"; tail -5 "$O/ab.err"; exit 1; }
    tail -1 "$O/ab.json" | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); p=r.get('parity',{}); c=r.get('corrected_camera',{}); print('r$r [$e]', r['ms_per_step'], r['frame_device_ms'], r['frame_wall_ms'], p.get('matches_reference'), c.get('ms_per_step'))"
  done
done
echo "=== done"
