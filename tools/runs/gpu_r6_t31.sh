#!/bin/bash
# r6 t31: 224x256 tiles on every grid where their rounds cost less (KUNGFU_CONV_T224=2) vs one/two-round grids only (1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2; do
  for m in 1 2; do
    KUNGFU_DEV_KNOBS=1 KUNGFU_CONV_T224=$m timeout -k 10 300 python bench.py --steps 30 --warmup 8 --comm-probe 0 > $O/r6t31_m${m}_$r.log 2>&1 || { tail -5 $O/r6t31_m${m}_$r.log; exit 1; }
    show $O/r6t31_m${m}_$r.log t224mode$m
  done
done
