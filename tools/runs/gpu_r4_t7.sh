#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread tests/test_gpu_convergence.py > $O/r4t7_conv.log 2>&1
grep -E "seed|stock|engine|last-|PASSED|FAILED|^E " $O/r4t7_conv.log | head -30
bash tools/runs/gpu_r4_t5.sh
