#!/bin/bash
# r6 t22: row-image 3x3 conv, two-workgroups-per-CU variants at 56x56
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_rows.py > $O/r6t22_test.log 2>&1; rc=$?
tail -3 $O/r6t22_test.log
[ $rc -eq 0 ] || exit $rc
SHAPES=0,1 timeout -k 10 200 python tools/bench_conv3x3_s1.py -1 2 20 21 22 24 25 > $O/r6t22_times.log 2>&1 || { tail -5 $O/r6t22_times.log; exit 1; }
cat $O/r6t22_times.log
