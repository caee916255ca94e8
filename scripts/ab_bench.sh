#!/usr/bin/env bash
# Interleaved bench.py A/B on one box: ROUNDS rounds of each --options variant (AB_OPTS, '|'-separated;
# an empty entry = the defaults). Prints ms_per_step, lone frame (device, wall) and footprint per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abb}
mkdir -p "$OUT"
IFS='|' read -r -a VARS <<< "${AB_OPTS:-|no_pairs=1}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for i in "${!VARS[@]}"; do
    v=${VARS[$i]}
    timeout -k 10 300 python bench.py --no-cpu-baseline --corrected-steps 0 ${BENCH_ARGS:-} --options "$v" > "$OUT/v${i}_r$r.json" 2> "$OUT/v${i}_r$r.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant '$v' round $r rc=$rc"; tail -3 "$OUT/v${i}_r$r.err"; exit $rc; fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(f\"{sys.argv[2]:32s} period {d['ms_per_step']:.3f} lone {d['frame_device_ms']:.3f} wall {d['frame_wall_ms']:.3f} hbm {d['hbm_footprint_bytes']/2**30:.2f} GiB parity {d.get('parity',{}).get('matches_reference')}\")" "$OUT/v${i}_r$r.json" "[$v]"
  done
done
