#!/bin/bash
# r6 t49: BERT-base + GNS regression check on one box: round-6 defaults vs the round-5 wgrad plan vs the main-stream bias colsum
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'])" $1 $2; }
A="--model bert_base --optimizer gns --steps 30 --warmup 8 --comm-probe 0"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/r6t49_def_$r.log 2>&1 || exit 1; show $O/r6t49_def_$r.log default
  KUNGFU_DEV_KNOBS=1 KUNGFU_WGRAD_PLAN=1 timeout -k 10 300 python bench.py $A > $O/r6t49_plan1_$r.log 2>&1 || exit 1; show $O/r6t49_plan1_$r.log wgrad_plan1
  timeout -k 10 300 python tools/bench_switch.py kungfu_amd.ops.linear:_BIAS_SIDE=False -- $A > $O/r6t49_bias_$r.log 2>&1 || exit 1; show $O/r6t49_bias_$r.log bias_main
done
