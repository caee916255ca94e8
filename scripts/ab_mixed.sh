#!/usr/bin/env bash
# Interleaved bench.py A/B over (library, options) variants on one box: AB_SPEC is a ';'-separated
# list of tag|lib|options (lib: "default" = the in-tree product, else a path to librt_mi355x.so);
# ROUNDS rounds. Prints period, lone frame (device), footprint and parity per run.
#   AB_SPEC="cur|default|;r04|scripts/_abl/r04/librt_mi355x.so|" ROUNDS=4 bash scripts/ab_mixed.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abm}; mkdir -p "$O"
IFS=';' read -r -a SPECS <<< "${AB_SPEC}"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for spec in "${SPECS[@]}"; do
    IFS='|' read -r tag lib opt <<< "$spec"
    if [ "$lib" = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --corrected-steps 0 ${BENCH_ARGS:-} --options "$opt" > "$O/${tag}_r$r.json" 2> "$O/${tag}_r$r.err"
    rc=$?; unset RT_LIB_PATH
    if [ $rc -ne 0 ]; then echo "FAIL $tag r$r rc=$rc"; tail -3 "$O/${tag}_r$r.err"; exit $rc; fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(f\"{sys.argv[2]:10s} period {d['ms_per_step']:.3f} lone {d['frame_device_ms']:.3f} hbm {d['hbm_footprint_bytes']/2**30:.2f} GiB parity {d['parity'].get('matches_reference')}\")" "$O/${tag}_r$r.json" "$tag"
  done
done
echo "=== done"
