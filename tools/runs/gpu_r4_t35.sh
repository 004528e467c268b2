#!/bin/bash
# NaN-filled uninitialised memory: which model paths read memory they never wrote? (eager, batch 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"].get("initial_loss"), d["config"].get("final_loss"))'; }
export KUNGFU_DEV_KNOBS=1
run() { local tag=$1; shift; timeout -k 10 300 env "$@" python tools/diag/nanfill_bench.py --batch 64 --steps 3 --warmup 2 --graph 0 ${ARGS} > $O/r4t35_$tag.log 2>&1; rc=$?; [ $rc -gt 1 ] && { tail -5 $O/r4t35_$tag.log; exit 1; }; echo "$tag rc=$rc $(tail -1 $O/r4t35_$tag.log | j)"; }
ARGS="--model vgg16" run vgg_layered KUNGFU_VGG_FUSED=0
ARGS="--model vgg16" run vgg_fused KUNGFU_VGG_FUSED=1
ARGS="--model resnet50" run resnet X=1
ARGS="--model inception_v3" run inception X=1
ARGS="--model bert_base --optimizer gns --batch 32" run bert X=1
