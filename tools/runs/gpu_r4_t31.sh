#!/bin/bash
# BERT-base + GNS: whole-step capture vs eager with the round-4 kernel set (A/B, one box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"), d["config"].get("final_loss"))'; }
for G in 0 1 0 1; do
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --graph $G --steps 30 --warmup 6 > $O/r4t31_bert_g$G.log 2>&1 || { tail -20 $O/r4t31_bert_g$G.log; exit 1; }
echo "bert graph=$G $(tail -1 $O/r4t31_bert_g$G.log | j)"
done
