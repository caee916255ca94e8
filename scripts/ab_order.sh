#!/usr/bin/env bash
# Interleaved A/B of render variants on one box (DESIGN.md §4.7 and later): config 3 bench lines,
# one per variant per round. VARIANTS: lines of "name lib options" (lib: default = the in-tree
# library, else a path from scripts/build_variant.sh; options: rt_options text or -).
#   VARIANTS=$'classes default -\nnatural default natural_order=1' ROUNDS=2 bash scripts/ab_order.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_order}
mkdir -p "$OUT"
V=${VARIANTS:-$'classes default -\nno_sky default no_sky=1\nnatural default natural_order=1'}
for r in $(seq 1 ${ROUNDS:-2}); do
  while read -r name lib opts; do
    [ -z "$name" ] && continue
    if [ "$lib" = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/$lib; fi
    o=""; [ "$opts" != "-" ] && o="--options $opts"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-dropin --corrected-steps 0 --steps ${STEPS:-20} $o ${BENCH_ARGS:-} > "$OUT/$name.$r.json" 2> "$OUT/$name.$r.err" || { echo "FAILED $name"; tail -5 "$OUT/$name.$r.err"; exit 1; }
    python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'period', r['ms_per_step'], 'lone', r['frame_device_ms'], 'wall', r['frame_wall_ms'], 'parity', r.get('parity',{}).get('matches_reference'))" "$OUT/$name.$r.json" "$name.$r"
  done <<< "$V"
done
unset RT_LIB_PATH
