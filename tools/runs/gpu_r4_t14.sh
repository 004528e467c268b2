#!/bin/bash
# BERT residual link with in-place addmm: tests + A/B bench; linear wgrad vs hipBLASLt microbench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
: tests passed in r4t14 first call

PYTHONPATH=$PWD timeout -k 10 200 python tools/bench_linear_wgrad.py > $O/r4t14_wgrad.log 2>&1; rc=$?; cat $O/r4t14_wgrad.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
for L in 1 0 1 0; do
KUNGFU_DEV_KNOBS=1 KUNGFU_RESIDUAL_LINK=$L timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t14_bert_l$L.log 2>&1 || { tail -20 $O/r4t14_bert_l$L.log; exit 1; }
echo "bert link=$L $(tail -1 $O/r4t14_bert_l$L.log | j)"
done
