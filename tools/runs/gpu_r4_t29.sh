#!/bin/bash
# BERT: linear weight-gradient split-K by f32 atomics into the slot vs the deterministic reduce (A/B, one box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("final_loss"))'; }
export KUNGFU_DEV_KNOBS=1
for A in 0 1 0 1; do
KUNGFU_LINEAR_WGRAD_ATOMICS=$A timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t29_bert_a$A.log 2>&1 || { tail -20 $O/r4t29_bert_a$A.log; exit 1; }
echo "bert atomics=$A $(tail -1 $O/r4t29_bert_a$A.log | j)"
done
