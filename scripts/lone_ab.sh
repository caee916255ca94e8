#!/usr/bin/env bash
# Lone-frame A/B of library builds: for ROUNDS rounds, each build in $LIBS ("default" = in-tree)
# runs scripts/ab_variants.py (lone config-3 frames, render kernels' span from HIP events, median
# of 5) at each spp in $SPPS. Prints one line per (round, spp, build).
#   LIBS="default scripts/_abl/x/librt_mi355x.so" SPPS="128 8" ROUNDS=3 bash scripts/lone_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-lone_ab}; mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for spp in ${SPPS:-128 8}; do
    for lib in ${LIBS:-default}; do
      n=$(echo "$lib" | tr -c 'a-zA-Z0-9' '_')
      if [ "$lib" = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/$lib; fi
      timeout -k 10 200 python scripts/ab_variants.py --rounds 5 --spp "$spp" --variants "exact:cull:s0" > "$O/r${r}_s${spp}_$n.log" 2>&1
      rc=$?; unset RT_LIB_PATH
      if [ $rc -ne 0 ]; then echo "FAIL $lib rc=$rc"; tail -3 "$O/r${r}_s${spp}_$n.log"; exit $rc; fi
      echo "r$r spp $spp $lib $(grep -o '"median_ms": [0-9.]*, "min_ms": [0-9.]*' "$O/r${r}_s${spp}_$n.log")"
    done
  done
done
echo "=== done"
