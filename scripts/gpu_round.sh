#!/usr/bin/env bash
# One GPU session: smoke -> parity tests -> bench -> rocprof kernel stats. Every GPU step has
# its own time limit; a crash/abort/timeout (exit >= 2 other than pytest's 1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    if [ $rc -eq 1 ] && [ "${STRICT:-0}" = 1 ]; then exit 1; fi
    return 0
}
for s in ${STEPS:-smoke pytest bench prof}; do
  case $s in
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    probe)  step probe 60 ./scripts/_bin/lds_oob_probe ;;
    new)    step new 600 python -u -m pytest ${NEW_TESTS:-tests} -m gpu -v --timeout 200 --timeout-method thread ;;
    rehearse) for n in ${REHEARSE_N:-2 4 8}; do
                step rehearse_n$n 600 python bench.py --rehearse-world $n --rehearse-gather --no-cpu-baseline --corrected-steps 0 ${BENCH_ARGS:-}
              done ;;
    pytest) step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ;;
    stock)  step stock 600 python bench.py --hw-queues 0 --no-cpu-baseline ${BENCH_ARGS:-} ;;
    bench)  step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    ab)     step ab 900 python scripts/ab_variants.py --rounds ${AB_ROUNDS:-5} --variants ${AB_VARIANTS:-exact:cull,fast:cull} ;;
    abl)    RT_LIB_PATH=$PWD/scripts/_abl/librt_mi355x.so step abl 900 python scripts/ab_variants.py --rounds ${AB_ROUNDS:-5} --variants ${AB_VARIANTS:-exact:cull,fast:cull} ;;
    prof)   step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --corrected-steps 0 ${BENCH_ARGS:-} ;;
  esac
done
echo "=== done"
