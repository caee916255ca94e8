set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g1
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1/smoke.log 2>&1 || { echo smoke fail $?; tail gpurun_out/g1/smoke.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g1/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/g1/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/g1/bench.log 2>&1 || exit $?
cat gpurun_out/g1/bench.log
RT_DEBUG_STATS=1 timeout -k 10 300 python scripts/ab_variants.py --rounds 2 --variants exact:cull > gpurun_out/g1/stats.log 2>&1 || exit $?
cat gpurun_out/g1/stats.log
