#!/bin/bash
# r6 t21: row-image 3x3 conv: numerics tests, then isolated timings vs the tap-wise variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_rows.py > $O/r6t21_test.log 2>&1; rc=$?
tail -25 $O/r6t21_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_conv3x3_s1.py -1 20 21 22 23 > $O/r6t21_times.log 2>&1 || { tail -5 $O/r6t21_times.log; exit 1; }
cat $O/r6t21_times.log
