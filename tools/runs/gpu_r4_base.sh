#!/bin/bash
# round-4 start: default benches + host-overhead measurement on a fresh box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r4a_resnet50.log 2>&1 || exit 1
tail -1 $O/r4a_resnet50.log
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r4a_bert.log 2>&1 || exit 1
tail -1 $O/r4a_bert.log
for M in resnet50 inception_v3; do
  timeout -k 10 300 python tools/diag/cpu_overhead.py $M > $O/r4a_cpu_$M.log 2>&1 || exit 1
  tail -6 $O/r4a_cpu_$M.log
done
