#!/bin/bash
# r6 t11: N > 1 defaults from measurement on the 1-GPU model of an 8-rank job
# (--emulate-comm 8 --emulate-ctas 16): Inception-v3 graph segments vs eager; f32 vs bf16 gradient wire
# dtype for ResNet-50 and BERT-base.  Two interleaved runs per arm.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("final_loss"), c.get("hip_graph"), c.get("comm",{}).get("comm_dtype"))'; }
run() {  # tag, args...
  local T=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 6 "$@" > $O/r6t11_$T.log 2>&1 || { tail -5 $O/r6t11_$T.log; exit 1; }
  echo "$T: $(tail -1 $O/r6t11_$T.log | j)"
}
E="--emulate-comm 8 --emulate-ctas 16"
for i in 1 2; do
  run incep_g1_$i --model inception_v3 $E --graph 1
  run incep_g0_$i --model inception_v3 $E --graph 0
done
for i in 1 2; do
  run r50_f32_$i $E --comm-dtype f32
  run r50_bf16_$i $E --comm-dtype bf16
done
for i in 1 2; do
  run bert_f32_$i --model bert_base --optimizer ssgd $E --comm-dtype f32
  run bert_bf16_$i --model bert_base --optimizer ssgd $E --comm-dtype bf16
done
