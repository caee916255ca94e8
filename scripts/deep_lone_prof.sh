#!/usr/bin/env bash
# Lone config-3 frames under rocprofv3 --kernel-trace, per library build in $LIBS ("default" =
# in-tree), ROUNDS interleaved rounds: the median duration of the lone deep launch
# (render_deep_kernel<..., 8>), of the main launch and of the accumulation parts.
#   LIBS="default scripts/_abl/x/librt_mi355x.so" ROUNDS=2 bash scripts/deep_lone_prof.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-deep_lone}; mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for lib in ${LIBS:-default}; do
    n=r${r}_$(echo "$lib" | tr -c 'a-zA-Z0-9' '_')
    if [ "$lib" = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/$lib; fi
    timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$O/$n" -o run -- \
      python3 scripts/ab_variants.py --rounds 5 --spp ${SPP:-128} --variants exact:cull:s0 > "$O/$n.log" 2>&1
    rc=$?; unset RT_LIB_PATH
    if [ $rc -ne 0 ]; then echo "FAIL $lib rc=$rc"; tail -3 "$O/$n.log"; exit $rc; fi
    python3 - "$O/$n" "$lib" <<'PY'
import csv, glob, statistics, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
def d(pred):
    v = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if pred(r["Kernel_Name"]))
    return (round(statistics.median(v), 1), round(v[0], 1), len(v)) if v else None
print(sys.argv[2], "deep8 us (median, min, n)", d(lambda k: "render_deep_kernel" in k and ", 8>" in k),
      "main", d(lambda k: "render_kernel<" in k and "true>" not in k), "acc", d(lambda k: "accumulate_kernel" in k))
PY
  done
done
echo "=== done"
