#!/usr/bin/env bash
# One rank's share of an N-way row split, rehearsed on one GPU (bench.py --rehearse-world N),
# next to the full frame at N = 1, for $CONFIG; JSON lines into gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-rehearse}
mkdir -p "$O"
C=${CONFIG:-c4}
timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --corrected-steps 0 --steps ${STEPS1:-5} --warmup 2 > "$O/${C}_n1.json" 2>"$O/${C}_n1.err" || exit $?
tail -1 "$O/${C}_n1.json"
for n in ${NS:-2 4 8}; do
  timeout -k 10 300 python bench.py --config $C --rehearse-world $n --no-cpu-baseline --corrected-steps 0 --steps ${STEPSN:-10} --warmup 3 > "$O/${C}_rehearse_n$n.json" 2>"$O/${C}_rehearse_n$n.err" || exit $?
  tail -1 "$O/${C}_rehearse_n$n.json" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$C n=$n', r['ms_per_step'], r['frame_latency_ms'], r['value'])"
done
echo "=== done"
