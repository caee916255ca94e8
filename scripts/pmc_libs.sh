#!/usr/bin/env bash
# Dynamic instruction counts of the render kernel per library build: one rocprofv3 --pmc pass
# (kernel trace only) over a short bench.py run per build in $LIBS; prints the mean per dispatch.
#   LIBS="default scripts/_abl/x/librt_mi355x.so" bash scripts/pmc_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-pmc_libs}
mkdir -p "$O"
export TMPDIR=/tmp
CNT=${PMC:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE}
for lib in ${LIBS:-default}; do
  n=$(echo "$lib" | tr -c 'a-zA-Z0-9' '_')
  if [ "$lib" = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/$lib; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d "$O/$n" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --corrected-steps 0 ${ARGS:-} > "$O/$n.log" 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $lib"; tail -5 "$O/$n.log"; exit $rc; fi
  python3 - "$O/$n" "$lib" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "render_kernel<" in r["Kernel_Name"] and "false, false>" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
by = collections.defaultdict(list)
for (_, c), v in per.items():
    by[c].append(v)
print(sys.argv[2], " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(by.items())))
PY
done
unset RT_LIB_PATH
echo "=== done"
