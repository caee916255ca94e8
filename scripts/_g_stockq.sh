#!/usr/bin/env bash
# the stock hardware-queue count (HIP's 4 -> 3 render streams) vs bench.py's 8, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/stockq; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for q in 8 4; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --corrected-steps 0 --hw-queues $q > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    tail -1 $O/b.json | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('r$r hwq=$q', r['ms_per_step'], r['frame_device_ms'], r['frame_wall_ms'], r['config']['hw_queues'], r['parity']['matches_reference'])"
  done
done
echo "=== done"
