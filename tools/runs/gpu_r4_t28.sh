#!/bin/bash
# VGG-16 layered path (KUNGFU_VGG_FUSED=0) under whole-step hipGraph: bisect the NaN
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph",{}).get("captured") if d["config"].get("hip_graph") else False, d["config"].get("final_loss"))'; }
export KUNGFU_DEV_KNOBS=1 KUNGFU_VGG_FUSED=0
run() { local tag=$1; shift; timeout -k 10 240 env "$@" python bench.py --model vgg16 --steps 8 --warmup 4 ${ARGS} > $O/r4t28_$tag.log 2>&1; rc=$?; [ $rc -gt 1 ] && { tail -5 $O/r4t28_$tag.log; exit 1; }; echo "$tag rc=$rc $(tail -1 $O/r4t28_$tag.log | j)"; }
ARGS="--graph 0 --batch 64" run eager_b64 X=1
ARGS="--graph 1 --batch 64" run graph_b64 X=1
ARGS="--graph 1 --batch 64 --lr 0.01" run graph_b64_lr01 X=1
ARGS="--graph 0 --batch 64" run eager_b64_fused KUNGFU_VGG_FUSED=1
ARGS="--graph 1 --batch 64" run graph_b64_fused KUNGFU_VGG_FUSED=1
ARGS="--graph 1 --batch 64" run graph_noconv_b64 KUNGFU_CONV3X3=0
ARGS="--graph 1 --batch 64" run graph_nowgrad_b64 KUNGFU_WGRAD=0
ARGS="--graph 1 --batch 64 --bf16-shadow 0" run graph_noshadow_b64 X=1
