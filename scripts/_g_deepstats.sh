#!/usr/bin/env bash
# STATS cycle shares and events of the deep launch alone (lone frame), shading records in LDS vs global
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/deepstats; mkdir -p $O; export TMPDIR=/tmp
for e in 1 0; do
  RT_DEEP_SHADE_LDS=$e RT_DEBUG_DEEP_ONLY=1 timeout -k 10 200 python scripts/stats_c3.py > $O/stats_deep_lds$e.json 2> $O/stats_deep_lds$e.err || { tail -5 $O/stats_deep_lds$e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/stats_deep_lds$e.json')); print('lds=$e', d['cycle_share'], d['wave_iters'], {k: d['events_per_iter'][k] for k in ('refill_trip','walk_skipped','dry_iter','hit','dielectric')})"
done
echo "=== done"
