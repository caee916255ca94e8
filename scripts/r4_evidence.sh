#!/usr/bin/env bash
# Round-4 evidence on one MI355X: GPU tests, the bench line, rocprofv3 kernel stats of the same
# command, PMC passes (scripts/pmc_round.sh), config 3 under a 4 GB workspace cap, the 2/4/8-way
# row-share rehearsals. Every step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r4_ev}
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -n 2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 400 python bench.py
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --no-cpu-baseline
TAG=${TAG:-r4_ev}/pmc step pmc 600 bash scripts/pmc_round.sh
step cap4g 400 python bench.py --no-cpu-baseline --corrected-steps 0 --options max_workspace_bytes=4294967296
step cap4g_ws1 400 python bench.py --no-cpu-baseline --corrected-steps 0 --options max_workspace_bytes=4294967296,workspaces_per_stream=1
for n in 2 4 8; do step rehearse_n$n 300 python bench.py --steps 40 --warmup 5 --rehearse-world $n --no-cpu-baseline --corrected-steps 0; done
echo "=== done"
