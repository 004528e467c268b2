#!/bin/bash
# r6 t34: kernel-trace profiles of the current ResNet-50 and BERT-base steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
bash tools/gpu_prof.sh ${TAG:-r6s2} resnet50 bert_base > $O/${TAG:-r6s2}_prof.log 2>&1 || { tail -5 $O/${TAG:-r6s2}_prof.log; exit 1; }
head -20 $O/${TAG:-r6s2}_resnet50_summary.md
