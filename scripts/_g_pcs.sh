#!/usr/bin/env bash
# PC sampling (stochastic, gfx950) over lone config-3 frames: where the waves stall
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-pcs}; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled 1 --pc-sampling-method ${METHOD:-stochastic} --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${IVAL:-1048576} --output-format csv -d $O/pcs -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --corrected-steps 0 > $O/pcs.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 $O/pcs.log; ls -la $O/pcs/* 2>/dev/null | head
find $O/pcs -name "*.csv" -size +50M -delete
echo "=== done"
