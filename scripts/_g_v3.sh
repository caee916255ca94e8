#!/usr/bin/env bash
# current tree vs head: parity subset, A/B (period, lone frame, 8-way), kernel durations
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${T:-v3}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
H=RT_LIB_PATH=$PWD/scripts/_abl/head/librt_mi355x.so
TAG=${T:-v3}/ab SETS1="-;$H${EXTRA1:-}" R1=${R1:-3} SETS8="-;$H" R8=${R8:-2} bash scripts/_g_ab.sh || exit 1
for e in cur head; do
  [ $e = head ] && export RT_LIB_PATH=$PWD/scripts/_abl/head/librt_mi355x.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$e -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --corrected-steps 0 > $O/kt_$e.log 2>&1 || exit 1
  python3 - $O/kt_$e <<'PY' || exit 1
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "render" in r["Name"] or "accum" in r["Name"]:
        print(sys.argv[1], r["Name"][:60], r["Calls"], r["AverageNs"])
PY
done
echo "=== done"
