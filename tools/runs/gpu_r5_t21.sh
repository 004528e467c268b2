#!/bin/bash
# r5 t21: ResNet-50 1x1 conv tile variants re-measured with the transposed epilogue (fwd + stats, dgrad modes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
VARIANTS=0,1,2,7,8 MODES=st,ab,bc timeout -k 10 600 python3 tools/bench_conv1x1_variants.py > $O/r5t21_conv1x1.txt 2>&1; rc=$?
grep -v amdgpu $O/r5t21_conv1x1.txt; exit $rc
