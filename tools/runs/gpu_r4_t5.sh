#!/bin/bash
# eager vs whole-step hipGraph (bench + host enqueue), configs 3/4 re-measured
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
for M in bert_base resnet50 inception_v3; do
  OPT=ssgd; [ $M = bert_base ] && OPT=gns
  for G in 0 1; do
    timeout -k 10 300 python bench.py --model $M --optimizer $OPT --steps 30 --warmup 6 --graph $G > $O/r4t5_${M}_g$G.log 2>&1 || { tail -20 $O/r4t5_${M}_g$G.log; exit 1; }
    echo "$M graph=$G $(tail -1 $O/r4t5_${M}_g$G.log | j)"
  done
done
for M in resnet50 inception_v3 bert_base; do
  for G in 0 1; do
    GRAPH=$G timeout -k 10 300 python tools/diag/cpu_overhead.py $M > $O/r4t5_cpu_${M}_g$G.log 2>&1 || { tail -20 $O/r4t5_cpu_${M}_g$G.log; exit 1; }
    echo "$M GRAPH=$G: $(grep 'host enqueue' $O/r4t5_cpu_${M}_g$G.log)"
  done
done
for o in sma pair; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 6 --optimizer $o > $O/r4t5_$o.log 2>&1 || { tail -20 $O/r4t5_$o.log; exit 1; }
  echo "$o $(tail -1 $O/r4t5_$o.log | j)"
done
