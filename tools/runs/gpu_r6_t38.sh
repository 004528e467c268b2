#!/bin/bash
# r6 t38: Inception-v3 and BERT-base with the round-6 weight-gradient plan rules vs round 5 (KUNGFU_WGRAD_PLAN)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2; do
  for m in 1 2; do
    KUNGFU_DEV_KNOBS=1 KUNGFU_WGRAD_PLAN=$m timeout -k 10 300 python bench.py --model inception_v3 --steps 20 --warmup 6 --comm-probe 0 > $O/r6t38_inc_m${m}_$r.log 2>&1 || { tail -5 $O/r6t38_inc_m${m}_$r.log; exit 1; }
    show $O/r6t38_inc_m${m}_$r.log inception_plan$m
  done
done
