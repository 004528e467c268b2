#!/bin/bash
# r6 t41: the RCCL-in-graph tests with thread-local capture, then the BERT linear wgrad sweep (t40)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rccl.py -k "hipgraph or graph" > $O/r6t41_test.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/r6t41_test.log | tail -6; [ $rc -eq 0 ] || exit $rc
bash tools/runs/gpu_r6_t40.sh
