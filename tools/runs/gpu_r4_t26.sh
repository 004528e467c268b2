#!/bin/bash
# VGG-16 default (eager again) + graph diagnosis, BERT default bench, emulated 8-rank ResNet-50 with graph
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"), d["config"].get("final_loss"), d.get("verify",{}).get("replicas_consistent"))'; }
timeout -k 10 300 python bench.py --model vgg16 --steps 20 --warmup 5 > $O/r4t26_vgg16.log 2>&1 || { tail -5 $O/r4t26_vgg16.log; exit 1; }
echo "vgg16 default $(tail -1 $O/r4t26_vgg16.log | j)"
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r4t26_bert.log 2>&1 || { tail -5 $O/r4t26_bert.log; exit 1; }
echo "bert default $(tail -1 $O/r4t26_bert.log | j)"
for C in 16 32; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --emulate-comm 8 --emulate-ctas $C > $O/r4t26_emu_c$C.log 2>&1 || { tail -5 $O/r4t26_emu_c$C.log; exit 1; }
echo "resnet50 emulate-8 ctas=$C $(tail -1 $O/r4t26_emu_c$C.log | j)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r4t26_resnet.log 2>&1 && echo "resnet50 $(tail -1 $O/r4t26_resnet.log | j)"
