#!/bin/bash
# r6 t39: stride-2 data-gradient tile sweep (current kernels) + stem bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/kungfu_amd/tuning/miopen
timeout -k 10 300 python -u tools/bench_dgrad_s2.py > $O/r6t39_s2.log 2>&1 || { tail -5 $O/r6t39_s2.log; exit 1; }
cat $O/r6t39_s2.log | grep -v "^/opt"
