#!/usr/bin/env bash
# A/B of an environment knob with bench.py: for each round, each value of $VAR in $VALUES, print
# ms_per_step, latency, Mrays/s, frame sha256 prefix. Every run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_env2}
mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for v in ${VALUES:-0 1}; do
    f="$O/r${r}_$v.log"
    env "${VAR:-RT_QUAD_ITEMS}=$v" timeout -k 10 200 python bench.py --no-cpu-baseline --corrected-steps 0 --digest ${ARGS:-} > "$f" 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $v"; tail -5 "$f"; exit $rc; fi
    grep '^{' "$f" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('r$r', '${VAR:-RT_QUAD_ITEMS}=$v', r['ms_per_step'], r['frame_latency_ms'], r['value'], r['frame_sha256'][:16], r['boxes_per_segment'], r['tests_per_segment'])"
  done
done
echo "=== done"
