#!/bin/bash
# r5 t38: qkv bias gradient from the attention backward's column sums: tests + same-box A/B (ops.attention._BIAS_LINK)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu.py tests/test_gpu_engine.py -k "attention or bert or linear or gemm" > $O/r5t38_pytest.log 2>&1
rc=$?; tail -1 $O/r5t38_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/r5t38_pytest.log | head -20; exit $rc; }
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() {
  timeout -k 10 300 python -c "
import sys, runpy
import kungfu_amd.ops.attention as at
at._BIAS_LINK = bool($1)
sys.argv = ['bench.py', '--model', 'bert_base', '--optimizer', 'gns', '--steps', '20', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > $O/r5t38_bert_b$1.log 2>&1 || { tail -5 $O/r5t38_bert_b$1.log; exit 1; }
  echo "attn bias link=$1: $(tail -1 $O/r5t38_bert_b$1.log | j)"
}
for r in 1 2; do run 0 && run 1 || exit 1; done
