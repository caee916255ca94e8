#!/usr/bin/env bash
# A/B of library builds on one GPU: for each round, for each build in $LIBS (paths to
# librt_mi355x.so, "default" = the in-tree product), run bench.py with $ARGS and print
# ms_per_step, single-frame latency and the frame's sha256 (every build must give the same bits).
# Every run has its own time limit; any failure ends the script.
#   LIBS="default scripts/_abl/x/librt_mi355x.so" ROUNDS=3 ARGS="..." bash scripts/ab_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_libs}
mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for lib in ${LIBS:-default}; do
    f="$O/r${r}_$(echo "$lib" | tr -c 'a-zA-Z0-9' '_').log"
    if [ "$lib" = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --corrected-steps 0 --digest ${ARGS:-} > "$f" 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $lib"; tail -5 "$f"; exit $rc; fi
    grep '^{' "$f" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('r$r', '$lib', r['ms_per_step'], r['frame_device_ms'], r['value'], r['parity'].get('frame_sha256','')[:16], r['parity'].get('matches_reference'), r['segments_per_primary'])"
  done
done
unset RT_LIB_PATH
echo "=== done"
