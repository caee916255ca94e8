#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-tl8}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --corrected-steps 0 --rehearse-world ${N:-8} --steps 40 > $O/prof.log 2>&1 || exit $?
python3 scripts/trace_timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --last 60 > $O/timeline.txt || exit $?
tail -8 $O/timeline.txt
echo "=== done"
