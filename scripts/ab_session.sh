#!/usr/bin/env bash
# One A/B session on the GPU box (each step under its own time limit; the first failure ends it):
#   lone frames of config 3 through scripts/ab_variants.py (option variants, interleaved rounds),
#   then bench.py frame streams and 8-way row-share rehearsals with and without each --options.
# AB_VARIANTS: ab_variants.py variants; BENCH_OPTS: space-separated --options strings ("-" = none).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
    [ $rc -eq 0 ] || exit $rc
}
if [ -n "${AB_VARIANTS:-}" ]; then
    run lone 600 python scripts/ab_variants.py --rounds "${AB_ROUNDS:-5}" --variants "$AB_VARIANTS"
fi
i=0
for o in ${BENCH_OPTS:-}; do
    i=$((i + 1))
    arg=(); [ "$o" = "-" ] || arg=(--options "$o")
    run "bench_$i" 400 python bench.py --no-cpu-baseline --corrected-steps 0 "${arg[@]}"
    [ "${REHEARSE:-0}" = 1 ] && run "r8_$i" 400 python bench.py --no-cpu-baseline --corrected-steps 0 --rehearse-world 8 --steps 40 "${arg[@]}"
done
echo "=== done"
