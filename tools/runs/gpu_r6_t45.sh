#!/bin/bash
# r6 t45: VGG-16 3x3 conv shapes on the tap-wise tiles vs the row-image kernel (plain epilogue)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for v in -1 0 1 2 7 8 20 21 22 24; do
  timeout -k 10 200 python -u tools/bench_vgg_conv.py --variant $v --iters 10 > $O/r6t45_v$v.log 2>&1 || { tail -3 $O/r6t45_v$v.log; exit 1; }
  echo "== v$v"; grep "H=" $O/r6t45_v$v.log
done
