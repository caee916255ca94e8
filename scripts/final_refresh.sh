#!/usr/bin/env bash
# Round-end refresh on one MI355X: smoke, parity tests, the bench line (with CPU baseline),
# rocprofv3 kernel stats of the same command, PMC passes, the other configs and the N-way
# rehearsals. Output under gpurun_out/$TAG; copy what is judged into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-final}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the script on any failure
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 400 python bench.py
cp "$O/bench.log" "$O/bench_c3.json"
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --no-cpu-baseline
TAG=${TAG:-final}/pmc step pmc 600 bash scripts/pmc_round.sh
for c in c2 c5 cuda c4; do step bench_$c 400 python bench.py --config $c --no-cpu-baseline --steps 3; done
step bench_c3corr 400 python bench.py --camera corrected --no-cpu-baseline --steps 3
step bench_c3fast 400 python bench.py --variant fast --no-cpu-baseline
for n in 2 4 8; do step rehearse_n$n 300 python bench.py --steps 40 --warmup 5 --rehearse-world $n; done
echo "=== done"
