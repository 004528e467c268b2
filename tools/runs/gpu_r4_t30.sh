#!/bin/bash
# VGG-16 under whole-step capture: NaN rate of the per-layer path vs eager vs the fused stack (batch 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"].get("final_loss"))'; }
export KUNGFU_DEV_KNOBS=1
run() { local tag=$1; shift; timeout -k 10 240 env "$@" python bench.py --model vgg16 --batch 64 --steps 8 --warmup 4 ${ARGS} > $O/r4t30_$tag.log 2>&1; rc=$?; [ $rc -gt 1 ] && { tail -5 $O/r4t30_$tag.log; exit 1; }; echo "$tag rc=$rc $(tail -1 $O/r4t30_$tag.log | j)"; }
for i in 1 2 3 4 5; do
ARGS="--graph 1" run layered_graph_$i KUNGFU_VGG_FUSED=0
ARGS="--graph 0" run layered_eager_$i KUNGFU_VGG_FUSED=0
ARGS="--graph 1" run fused_graph_$i KUNGFU_VGG_FUSED=1
done
