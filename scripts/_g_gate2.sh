#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/gate2; mkdir -p $O; export TMPDIR=/tmp
H=$PWD/scripts/_abl/head/librt_mi355x.so
TAG=gate2/c3 SETS="-;RT_LIB_PATH=$H" ROUNDS=5 bash scripts/ab_env3.sh || exit 1
TAG=gate2/s4 SETS="-;RT_LIB_PATH=$H" ROUNDS=3 ARGS="--rehearse-world 4" bash scripts/ab_env3.sh || exit 1
timeout -k 10 300 python bench.py --hw-queues 0 --no-cpu-baseline > $O/stock.json 2> $O/stock.err || exit 1
tail -1 $O/stock.json | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('stock queues', r['config']['hw_queues_env'], r['frames_in_flight'], r['ms_per_step'], r['frame_device_ms'], r['frame_wall_ms'])"
echo "=== done"
