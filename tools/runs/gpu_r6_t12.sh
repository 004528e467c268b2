#!/bin/bash
# r6 t12: side-stream read/in-place-write fix (linear gemm A/B diag + gemm tests), then stem tests + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 240 python -u tools/diag/linear_gemm_ab.py --lr 1e-4 --steps 2 > $O/r6t12_ab.log 2>&1 || { tail -5 $O/r6t12_ab.log; exit 1; }
grep step $O/r6t12_ab.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -q --timeout 120 --timeout-method thread > $O/r6t12_gemm.log 2>&1
grep -E "FAILED|passed|failed" $O/r6t12_gemm.log | tail -6
bash tools/runs/gpu_r6_t10.sh
