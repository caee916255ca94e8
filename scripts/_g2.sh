set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/g2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python scripts/ab_variants.py --rounds 5 --variants exact:cull5:t0,exact:cull5:t8,exact:cull6:t0,exact:cull6:t8,exact:cull6:t15 > $O/ab.log 2>&1 || exit $?
cat $O/ab.log
