#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
SEEDS=1,2,3 PEAKS=0.2,0.05 timeout -k 10 900 python tools/diag/conv_ablation.py stock ssgd fusedbn engine > $O/r4t6_ablation.log 2>&1; grep -E "MEAN|Error" $O/r4t6_ablation.log
