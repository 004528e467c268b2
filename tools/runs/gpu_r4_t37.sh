#!/bin/bash
# VGG-16 per-layer path: captured vs eager final loss per component swap (which one makes the replay differ?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], repr(d["config"].get("final_loss")))'; }
export KUNGFU_DEV_KNOBS=1 KUNGFU_VGG_FUSED=0
run() { local tag=$1; shift; timeout -k 10 240 env "$@" python bench.py --model vgg16 --batch 64 --steps 8 --warmup 4 ${ARGS} > $O/r4t37_$tag.log 2>&1; rc=$?; [ $rc -ge 124 ] && { tail -5 $O/r4t37_$tag.log; exit 1; }; echo "$tag rc=$rc $(tail -1 $O/r4t37_$tag.log | j)"; }
for V in base:X=1 noconv:KUNGFU_CONV3X3=0 nowgrad:KUNGFU_WGRAD=0 noshadow:SHADOW=0; do
  T=${V%%:*}; E=${V#*:}; EXTRA=""; [ $T = noshadow ] && EXTRA="--bf16-shadow 0"
  ARGS="--graph 0 $EXTRA" run ${T}_eager $E
  ARGS="--graph 1 $EXTRA" run ${T}_graph1 $E
  ARGS="--graph 1 $EXTRA" run ${T}_graph2 $E
done
