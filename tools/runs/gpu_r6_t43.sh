#!/bin/bash
# r6 t43: VGG-16 3x3 weight-gradient variants x splits under the round-6 plan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/kungfu_amd/tuning/miopen
timeout -k 10 800 python -u tools/bench_vgg_wgrad.py > $O/r6t43_vgg_wgrad.log 2>&1 || { tail -5 $O/r6t43_vgg_wgrad.log; exit 1; }
grep "N=" $O/r6t43_vgg_wgrad.log
