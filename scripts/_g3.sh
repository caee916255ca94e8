set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/g3; mkdir -p $O
export TMPDIR=/tmp
RT_VERBOSE=1 timeout -k 10 600 python scripts/ab_variants.py --rounds 5 --variants exact:cull5:t0:L0,exact:cull5:t0:L1,exact:cull6:t15:L0,exact:cull6:t15:L1 > $O/ab.log 2>&1 || exit $?
grep -v "^\[rt\]" $O/ab.log; grep "^\[rt\]" $O/ab.log | sort | uniq -c
RT_DEBUG_STATS=1 timeout -k 10 300 python scripts/ab_variants.py --rounds 1 --variants exact:cull5:t0,exact:cull6:t15 > $O/stats.log 2>&1 || exit $?
cat $O/stats.log
