#!/bin/bash
# r5 t35: A/B on one box -- FC2 data gradient + GELU backward fused (ops.linear._GELU_GEMM) vs hipBLASLt + gelu_bwd_colsum
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() {
  timeout -k 10 300 python -c "
import sys, runpy
import kungfu_amd.ops.linear as lin
lin._GELU_GEMM = bool($1)
sys.argv = ['bench.py', '--model', 'bert_base', '--optimizer', 'gns', '--steps', '20', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > $O/r5t35_bert_gg$1.log 2>&1 || { tail -5 $O/r5t35_bert_gg$1.log; exit 1; }
  echo "gelu_gemm=$1: $(tail -1 $O/r5t35_bert_gg$1.log | j)"
}
for r in 1 2; do run 0 && run 1 || exit 1; done
