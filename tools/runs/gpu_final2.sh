#!/bin/bash
# round-end rehearsal + the other conv models' benches + ResNet-50 profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash tools/gpu_final.sh r3z2 || exit 1
for M in inception_v3 vgg16; do
  timeout -k 10 300 python bench.py --model $M --steps 20 --warmup 5 > $O/r3z2_$M.log 2>&1 || exit 1
  echo "$M $(tail -1 $O/r3z2_$M.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
bash tools/gpu_prof.sh r3z2 resnet50 inception_v3 | grep -E "kernel sum"
