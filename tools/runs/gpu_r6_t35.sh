#!/bin/bash
# r6 t35: re-sweep the conv tile variants on the ResNet-50 1x1 and 3x3 shapes (current kernels) against the defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
VARIANTS=-1,0,1,2,7,8 MODES=st,ab,bc timeout -k 10 400 python tools/bench_conv1x1_variants.py > $O/r6t35_k1.log 2>&1 || { tail -5 $O/r6t35_k1.log; exit 1; }
cat $O/r6t35_k1.log | grep H=
KS3=1 VARIANTS=-1,0,1,2,7,8 MODES=st,bc timeout -k 10 400 python tools/bench_conv1x1_variants.py > $O/r6t35_k3.log 2>&1 || { tail -5 $O/r6t35_k3.log; exit 1; }
cat $O/r6t35_k3.log | grep H=
