#!/bin/bash
# r5 t36: A/B on one box -- MLM logits GEMM on gemm.hip gemm_nt_ld ("ours") vs hipBLASLt into the padded rows ("blas")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() {
  timeout -k 10 300 python -c "
import sys, runpy
import kungfu_amd.ops.vocab as vb
vb._FWD = '$1'
sys.argv = ['bench.py', '--model', 'bert_base', '--optimizer', 'gns', '--steps', '20', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > $O/r5t36_bert_$1.log 2>&1 || { tail -5 $O/r5t36_bert_$1.log; exit 1; }
  echo "vocab fwd=$1: $(tail -1 $O/r5t36_bert_$1.log | j)"
}
for r in 1 2; do run ours && run blas || exit 1; done
