#!/bin/bash
# r5 t32: ResNet-50 / Inception-v3 with the conv weight gradients on the side stream (A/B, same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() {  # $1 = side (0/1), $2 = model
  timeout -k 10 300 python -c "
import sys, runpy
import kungfu_amd.parallel.mixed as m
m.SideStream.enabled = bool($1)
sys.argv = ['bench.py', '--model', '$2', '--steps', '30', '--warmup', '8']
runpy.run_path('bench.py', run_name='__main__')
" > $O/r5t32_$2_s$1.log 2>&1 || { tail -5 $O/r5t32_$2_s$1.log; exit 1; }
  echo "$2 side=$1: $(tail -1 $O/r5t32_$2_s$1.log | j)"
}
for r in 1 2; do
  run 0 resnet50 && run 1 resnet50 || exit 1
done
run 0 inception_v3 && run 1 inception_v3
