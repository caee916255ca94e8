#!/usr/bin/env bash
# A/B of an environment knob on one GPU: for each round, for each value of $VAR in $VALUES,
# run each bench.py argument set in $CASES (';'-separated) and print one summary line.
# Every run has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_env}
mkdir -p "$O"
IFS=';' read -ra cases <<< "${CASES:---no-cpu-baseline;--rehearse-world 8 --steps 40 --warmup 5}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in ${VALUES:-1 2}; do
    for c in "${cases[@]}"; do
      f="$O/r${r}_${v}_$(echo "$c" | tr -c 'a-z0-9' '_').log"
      env "${VAR:-RT_WS_PER_STREAM}=$v" timeout -k 10 200 python bench.py $c > "$f" 2>&1
      rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $v $c"; tail -5 "$f"; exit $rc; fi
      grep '^{' "$f" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$r', '$v', '$c', r['ms_per_step'], r['frame_latency_ms'], r['roofline']['kernel_avg_ms'], r['value'])"
    done
  done
done
echo "=== done"
