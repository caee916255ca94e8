#!/usr/bin/env bash
# isolated-sphere shortcut: GPU tests, then A/B RT_ISO on config 3, the 8-way share and config 5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/iso; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k isolated --timeout 200 --timeout-method thread > $O/pytest_iso.log 2>&1; rc=$?
tail -3 $O/pytest_iso.log
[ $rc -eq 0 ] || exit $rc
TAG=iso/c3 SETS="-;RT_ISO=0" ROUNDS=3 bash scripts/ab_env3.sh || exit 1
TAG=iso/s8 SETS="-;RT_ISO=0" ROUNDS=2 ARGS="--rehearse-world 8" bash scripts/ab_env3.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
TAG=iso/c5 SETS="-;RT_ISO=0" ROUNDS=1 ARGS="--config c5 --steps 3" bash scripts/ab_env3.sh || exit 1
echo "=== done"
