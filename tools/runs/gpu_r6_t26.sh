#!/bin/bash
# r6 t26: where gemm.hip stands against hipBLASLt on the BERT-base products
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/bench_gemm_nt.py > $O/r6t26_gemm.log 2>&1 || { tail -5 $O/r6t26_gemm.log; exit 1; }
cat $O/r6t26_gemm.log
