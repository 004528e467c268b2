#!/bin/bash
# GELU forward kernel: test + BERT A/B (same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu.py -k "gelu_forward" > $O/r4t20_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/r4t20_pytest.log | head -30; [ $rc -eq 0 ] || exit $rc
for G in 1 0 1 0; do
KUNGFU_DEV_KNOBS=1 KUNGFU_GELU_FWD=$G timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t20_bert_g$G.log 2>&1 || { tail -20 $O/r4t20_bert_g$G.log; exit 1; }
echo "bert gelu_fwd=$G $(tail -1 $O/r4t20_bert_g$G.log | j)"
done
for M in resnet50 inception_v3; do
  timeout -k 10 300 python bench.py --model $M --steps 30 --warmup 6 > $O/r4t20_$M.log 2>&1 || { tail -20 $O/r4t20_$M.log; exit 1; }
  echo "$M $(tail -1 $O/r4t20_$M.log | j)"
done
