#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/nb; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "isolated or cluster_culling or golden_render_f32" --timeout 200 --timeout-method thread > $O/pytest_iso.log 2>&1; rc=$?
tail -3 $O/pytest_iso.log
[ $rc -eq 0 ] || exit $rc
TAG=nb/c3 SETS="-;RT_ISO_NB=0" ROUNDS=3 bash scripts/ab_env3.sh || exit 1
TAG=nb/s8 SETS="-;RT_ISO_NB=0" ROUNDS=2 ARGS="--rehearse-world 8" bash scripts/ab_env3.sh || exit 1
RT_DEBUG_DEEP_ONLY=1 timeout -k 10 200 python scripts/stats_c3.py > $O/stats_deep.json 2> $O/stats_deep.err || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
echo "=== done"
