#!/usr/bin/env bash
# deep launch with its shading records in LDS: parity subset, A/B (lone frame + period), deep-launch duration
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/dshade; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
TAG=dshade/ab SETS1="-;RT_DEEP_SHADE_LDS=0" R1=3 SETS8="-;RT_DEEP_SHADE_LDS=0" R8=2 bash scripts/_g_ab.sh || exit 1
for e in 1 0; do
  RT_DEEP_SHADE_LDS=$e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$e -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --corrected-steps 0 > $O/kt$e.log 2>&1 || exit 1
  python3 - $O/kt$e <<'PY' || exit 1
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "render" in r["Name"] or "accum" in r["Name"]:
        print(sys.argv[1], r["Name"][:60], r["Calls"], r["AverageNs"])
PY
done
echo "=== done"
