#!/bin/bash
# BERT: residual-gradient link, no materialised zero weight grads, embedding kernel sweep; tests, bench, profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_embedding.py tests/test_gpu.py tests/test_gpu_engine.py \
  -k "embedding or bert or graphed or linear" > $O/r4t13_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/r4t13_pytest.log | head -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/diag/bert_fills.py > $O/r4t13_fills.log 2>&1; rc=$?; head -30 $O/r4t13_fills.log | cut -c1-200; grep "embedding grad" $O/r4t13_fills.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t13_bert$i.log 2>&1 || { tail -20 $O/r4t13_bert$i.log; exit 1; }
echo "bert $(tail -1 $O/r4t13_bert$i.log | j)"
done
KUNGFU_DEV_KNOBS=1 KUNGFU_RESIDUAL_LINK=0 timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t13_bert_nolink.log 2>&1 || { tail -20 $O/r4t13_bert_nolink.log; exit 1; }
echo "bert no-link $(tail -1 $O/r4t13_bert_nolink.log | j)"
bash tools/gpu_prof.sh r4t13 bert_base
