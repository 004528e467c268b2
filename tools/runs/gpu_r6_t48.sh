#!/bin/bash
# r6 t48: all four benchmark models on one box at the driver's 20 / 5 configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['config']['initial_loss'],d['config']['final_loss'])" $1 $2; }
for M in resnet50 inception_v3 vgg16; do
  timeout -k 10 300 python bench.py --model $M --gpus 1 --steps 20 --warmup 5 > $O/r6t48_$M.log 2>&1 || { tail -5 $O/r6t48_$M.log; exit 1; }
  show $O/r6t48_$M.log $M
done
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --gpus 1 --steps 20 --warmup 5 > $O/r6t48_bert.log 2>&1 || { tail -5 $O/r6t48_bert.log; exit 1; }
show $O/r6t48_bert.log bert_base_gns
