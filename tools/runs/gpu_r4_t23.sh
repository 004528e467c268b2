#!/bin/bash
# BERT eager vs whole-step graph (GNS), after the round-4 BERT kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"), d["config"].get("final_loss"), d["config"].get("gradient_noise_scale"))'; }
for G in 1 0 1 0; do
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 --graph $G > $O/r4t23_bert_g$G.log 2>&1 || { tail -20 $O/r4t23_bert_g$G.log; exit 1; }
echo "bert graph=$G $(tail -1 $O/r4t23_bert_g$G.log | j)"
done
GRAPH=1 timeout -k 10 300 python tools/diag/cpu_overhead.py bert_base > $O/r4t23_cpu_bert_g1.log 2>&1 && grep "host enqueue" $O/r4t23_cpu_bert_g1.log
GRAPH=0 timeout -k 10 300 python tools/diag/cpu_overhead.py bert_base > $O/r4t23_cpu_bert_g0.log 2>&1 && grep "host enqueue" $O/r4t23_cpu_bert_g0.log
