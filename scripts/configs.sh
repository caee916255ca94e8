#!/usr/bin/env bash
# Bench lines of the other configurations (no CPU baseline): config 2, 5, the cuda_impl preset,
# config 3 with the fast kernel. JSON lines into gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-configs}
mkdir -p "$O"
for c in "c2" "c5 --steps 5" "cuda" "c3 --variant fast"; do
  n=$(echo "$c" | tr -c 'a-z0-9' '_')
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --corrected-steps 0 > "$O/$n.json" 2> "$O/$n.err" || exit $?
  tail -1 "$O/$n.json" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$c', r['ms_per_step'], r['frame_latency_ms'], r['value'], r['segments_per_primary'])"
done
echo "=== done"
