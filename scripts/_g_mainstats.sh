#!/usr/bin/env bash
# STATS cycle shares and events per wave iteration of a config-3 frame (main launch and deep launch), current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mainstats; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python scripts/stats_c3.py > $O/stats_frame.json 2> $O/stats_frame.err || { tail -5 $O/stats_frame.err; exit 1; }
RT_DEBUG_DEEP_ONLY=1 timeout -k 10 200 python scripts/stats_c3.py > $O/stats_deep.json 2> $O/stats_deep.err || { tail -5 $O/stats_deep.err; exit 1; }
python3 -c "
import json
for f in ('frame', 'deep'):
    d = json.load(open('$O/stats_' + f + '.json'))
    print(f, d['wave_iters'], round(d['live_lanes_per_iter'], 1) if 'live_lanes_per_iter' in d else '', d['cycle_share'])
    print(f, {k: round(v, 3) for k, v in d['events_per_iter'].items()})
"
echo "=== done"
