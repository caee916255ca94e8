#!/usr/bin/env bash
# The round's profile set on the committed build: the bench line, rocprofv3 kernel-trace stats
# of the same command, the per-dispatch timeline (frame stream + lone frames), stock queues.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r3prof}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --corrected-steps 0 > $O/prof.log 2>&1 || exit $?
python3 scripts/trace_timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --last 40 > $O/timeline.txt || exit $?
tail -4 $O/timeline.txt
timeout -k 10 300 python bench.py --hw-queues 0 --no-cpu-baseline > $O/bench_stock.json 2> $O/bench_stock.err || exit $?
tail -1 $O/bench_stock.json | cut -c1-300
echo "=== done"
