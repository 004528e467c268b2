#!/bin/bash
# r6 t18 (session 2 re-entry): driver-exact bench on HEAD + kernel-trace profiles of ResNet-50 and BERT-base
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/r6t18_bench.log 2>&1 || { tail -5 $O/r6t18_bench.log; exit 1; }
tail -1 $O/r6t18_bench.log
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r6t18_bert.log 2>&1 || { tail -5 $O/r6t18_bert.log; exit 1; }
tail -1 $O/r6t18_bert.log
bash tools/gpu_prof.sh r6t18 resnet50 bert_base > $O/r6t18_prof.log 2>&1 || { tail -5 $O/r6t18_prof.log; exit 1; }
cat $O/r6t18_prof.log
