#!/usr/bin/env bash
# STATS events of the full config-3 frame and of its deep launch alone, and the rocprof
# per-dispatch timeline of lone frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-diag}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python scripts/stats_c3.py > $O/stats_frame.json 2> $O/stats_frame.err || exit $?
RT_DEBUG_DEEP_ONLY=1 timeout -k 10 200 python scripts/stats_c3.py > $O/stats_deep.json 2> $O/stats_deep.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --corrected-steps 0 --steps 5 > $O/prof.log 2>&1 || exit $?
python3 scripts/trace_timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --last 40 > $O/timeline.txt || exit $?
echo "=== done"
