#!/bin/bash
# ResNet-50 with an emulated 8-rank all-reduce per bucket: whole-step capture vs eager (A/B, one box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph",{}) and d["config"]["hip_graph"].get("captured"))'; }
for G in 0 1 0 1; do
for C in 16 32; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph $G --emulate-comm 8 --emulate-ctas $C > $O/r4t33_g${G}_c$C.log 2>&1 || { tail -5 $O/r4t33_g${G}_c$C.log; exit 1; }
echo "emulate-8 graph=$G ctas=$C $(tail -1 $O/r4t33_g${G}_c$C.log | j)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph $G > $O/r4t33_g${G}_base.log 2>&1 || { tail -5 $O/r4t33_g${G}_base.log; exit 1; }
echo "no emulation graph=$G $(tail -1 $O/r4t33_g${G}_base.log | j)"
done
