#!/bin/bash
# r6 t16: the new N > 1 defaults in effect (emulated 8 ranks: Inception eager, bf16 wire incl. GNS), then a
# current VGG-16 kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("final_loss"), c.get("hip_graph"), c.get("comm",{}).get("comm_dtype"))'; }
timeout -k 10 300 python bench.py --model inception_v3 --emulate-comm 8 --steps 10 --warmup 4 > $O/r6t16_incep.log 2>&1 || { tail -5 $O/r6t16_incep.log; exit 1; }
echo "incep emu8 default: $(tail -1 $O/r6t16_incep.log | j)"
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --emulate-comm 8 --steps 10 --warmup 4 > $O/r6t16_bert.log 2>&1 || { tail -5 $O/r6t16_bert.log; exit 1; }
echo "bert gns emu8 default: $(tail -1 $O/r6t16_bert.log | j)"
bash tools/gpu_prof.sh r6x vgg16
