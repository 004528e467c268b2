#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/diag/conv_ablation.py > $O/r4t4_ablation.log 2>&1; grep -E "loss|Error|error" $O/r4t4_ablation.log | tail -20
bash tools/runs/gpu_r4_pmc.sh 2>&1 | tail -30
