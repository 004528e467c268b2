#!/bin/bash
# r6 t36: weight-gradient tile/split sweep on every ResNet-50 shape (current kernels) vs the planned defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/kungfu_amd/tuning/miopen
timeout -k 10 900 python -u tools/bench_wgrad.py --sweep > $O/r6t36_wgrad.log 2>&1 || { tail -5 $O/r6t36_wgrad.log; exit 1; }
cat $O/r6t36_wgrad.log | cut -c1-60,100-400
