#!/bin/bash
# r5 t39: LayerNorm backward grid (rows per wave 8 / 4 / 2) A/B on one box, BERT-base + GNS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() {
  timeout -k 10 300 python -c "
import sys, runpy
from kungfu_amd._lib import hip
hip().set_layernorm_bwd_rows_per_wave($1)
sys.argv = ['bench.py', '--model', 'bert_base', '--optimizer', 'gns', '--steps', '20', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > $O/r5t39_bert_r$1.log 2>&1 || { tail -5 $O/r5t39_bert_r$1.log; exit 1; }
  echo "ln bwd rows/wave=$1: $(tail -1 $O/r5t39_bert_r$1.log | j)"
}
for r in 1 2; do run 8 && run 4 && run 2 || exit 1; done
