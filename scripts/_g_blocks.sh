#!/usr/bin/env bash
# 8-way share: every rank's rows, interleaved (every 8th row) vs one contiguous block
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/blocks; mkdir -p $O; export TMPDIR=/tmp
for lay in "" "--rehearse-blocks"; do
  for r in 0 1 2 3 4 5 6 7; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --corrected-steps 0 --rehearse-world 8 --rehearse-rank $r $lay > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    tail -1 $O/b.json | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('[$lay] rank $r', r['ms_per_step'], r['frame_device_ms'], r['segments_per_primary'], r['boxes_per_segment'], r['tests_per_segment'], r['parity'].get('matches_reference'))"
  done
done
echo "=== done"
