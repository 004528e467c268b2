#!/bin/bash
# r5 t13: row-image wgrad variants 6 / 8-12 after the split-group dense reduce: numerics + per-shape timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wgrad_rows.py > $O/r5t13_pytest.log 2>&1
rc=$?; tail -1 $O/r5t13_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_inception_wgrad.py > $O/r5t13_wgrad.txt 2>&1 || exit 1
grep -E "rows|weighted" $O/r5t13_wgrad.txt
