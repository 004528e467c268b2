#!/bin/bash
# r5 t30: BERT linear weight gradients on the side stream (A/B, same box) + tests of the linear path
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for r in 1 2; do
for S in 0 1; do
  KUNGFU_LINEAR_WGRAD_SIDE=$S timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r5t30_bert_s$S.log 2>&1 || { tail -5 $O/r5t30_bert_s$S.log; exit 1; }
  echo "side=$S: $(tail -1 $O/r5t30_bert_s$S.log | j)"
done
done
KUNGFU_LINEAR_WGRAD_SIDE=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_engine.py -k "linear or bert or gns" > $O/r5t30_pytest.log 2>&1
rc=$?; tail -1 $O/r5t30_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/r5t30_pytest.log | head -20; exit $rc; }
