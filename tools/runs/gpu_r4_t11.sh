#!/bin/bash
# BERT with the scatter-add embedding gradient: eager vs whole-step graph (bench + host enqueue),
# graphed BERT bit-identity test, configs 3/4, ResNet default, BERT + ResNet profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
timeout -k 10 900 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_embedding.py tests/test_gpu_engine.py -k "embedding or graphed or self_launch or whole_step_graph or hipgraph or cta_budget" > $O/r4t11_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/r4t11_pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for G in 0 1; do
  timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 --graph $G > $O/r4t11_bert_g$G.log 2>&1 || { tail -20 $O/r4t11_bert_g$G.log; exit 1; }
  echo "bert graph=$G $(tail -1 $O/r4t11_bert_g$G.log | j)"
  GRAPH=$G timeout -k 10 300 python tools/diag/cpu_overhead.py bert_base > $O/r4t11_cpu_bert_g$G.log 2>&1 || { tail -20 $O/r4t11_cpu_bert_g$G.log; exit 1; }
  echo "bert GRAPH=$G: $(grep 'host enqueue' $O/r4t11_cpu_bert_g$G.log)"
done
for o in sma pair; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 6 --optimizer $o > $O/r4t11_$o.log 2>&1 || { tail -20 $O/r4t11_$o.log; exit 1; }
  echo "$o $(tail -1 $O/r4t11_$o.log | j)"
done
timeout -k 10 300 python bench.py --steps 30 --warmup 6 > $O/r4t11_resnet50.log 2>&1 && echo "resnet50 $(tail -1 $O/r4t11_resnet50.log | j)" || exit 1
bash tools/gpu_prof.sh r4t11 bert_base resnet50
