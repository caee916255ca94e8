#!/usr/bin/env bash
# Config-3 row shares rehearsed on one GPU (bench.py --rehearse-world N, rank 0's rows) with and
# without a rocprofv3 kernel trace, for the 1/2/4/8-way scaling analysis.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r3tl}
mkdir -p "$O"
export TMPDIR=/tmp
for n in ${NS:-8 4}; do
  timeout -k 10 200 python bench.py --rehearse-world $n --no-cpu-baseline --corrected-steps 0 --steps 20 --warmup 3 ${EXTRA:-} > "$O/c3_n$n.json" 2> "$O/c3_n$n.err" || exit $?
  tail -1 "$O/c3_n$n.json" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('n=$n', r['ms_per_step'], r['frame_device_ms'], r['parity'].get('matches_reference'))"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tl$n" -o run -- python3 bench.py --rehearse-world $n --no-cpu-baseline --corrected-steps 0 --steps 20 --warmup 3 ${EXTRA:-} > "$O/tl$n.log" 2>&1 || exit $?
  python scripts/trace_timeline.py $(find "$O/tl$n" -name "*kernel_trace.csv" | head -1) > "$O/tl$n.txt" || exit $?
  tail -3 "$O/tl$n.txt"
done
echo "=== done"
