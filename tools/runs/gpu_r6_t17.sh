#!/bin/bash
# r6 t17: wire dtype A/B for Inception-v3 (eager) and BERT-base + GNS at emulated 8 ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("final_loss"), c.get("hip_graph"), c.get("comm",{}).get("comm_dtype"))'; }
run() {
  local T=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 6 "$@" > $O/r6t17_$T.log 2>&1 || { tail -5 $O/r6t17_$T.log; exit 1; }
  echo "$T: $(tail -1 $O/r6t17_$T.log | j)"
}
E="--emulate-comm 8 --emulate-ctas 16"
for i in 1 2; do
  run incep_f32_$i --model inception_v3 $E --comm-dtype f32
  run incep_bf16_$i --model inception_v3 $E --comm-dtype bf16
done
run bertgns_f32 --model bert_base --optimizer gns $E --comm-dtype f32
run bertgns_bf16 --model bert_base --optimizer gns $E --comm-dtype bf16
