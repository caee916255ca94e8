#!/usr/bin/env bash
# A/B against the round-3 tree (a copy built in scripts/_abl/r03, not tracked): its bench.py,
# then this tree's with each --options string, then round 3 again (interleaved for box noise).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/${TAG:-abr03}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --corrected-steps 0 ${EXTRA:-}"
r03() {
    echo "=== r03 $1 ($(date +%T))"
    (cd scripts/_abl/r03 && timeout -k 10 400 python bench.py $ARGS > "$OUT/r03_$1.log" 2>&1) || { tail -5 "$OUT/r03_$1.log"; exit 1; }
    tail -c 300 "$OUT/r03_$1.log" | head -c 0; python3 -c "import json,sys; r=json.loads(open('$OUT/r03_$1.log').read().strip().splitlines()[-1]); print('r03', r['ms_per_step'], r['frame_device_ms'], r['value'])"
}
r03 a
i=0
for o in ${BENCH_OPTS:--}; do
    i=$((i + 1))
    arg=(); [ "$o" = "-" ] || arg=(--options "$o")
    echo "=== r04 $o ($(date +%T))"
    timeout -k 10 400 python bench.py $ARGS "${arg[@]}" > "$OUT/r04_$i.log" 2>&1 || { tail -5 "$OUT/r04_$i.log"; exit 1; }
    python3 -c "import json,sys; r=json.loads(open('$OUT/r04_$i.log').read().strip().splitlines()[-1]); print('r04 $o', r['ms_per_step'], r['frame_device_ms'], r['value'], r['pass_samples'])"
done
r03 b
echo "=== done"
