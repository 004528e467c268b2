#!/bin/bash
# r5 t24: MLM head products (decoder forward / dgrad / wgrad / bias colsum) on hipBLASLt variants vs gemm.hip
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/bench_mlm_head.py > $O/r5t24_mlm.log 2>&1; rc=$?
cat $O/r5t24_mlm.log; exit $rc
