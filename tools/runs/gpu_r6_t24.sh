#!/bin/bash
# r6 t24: ResNet-50 A/B of the row-image 3x3 conv at 56x56 (KUNGFU_CONV_ROWS dev knob), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 8 --comm-probe 0 > $O/r6t24_base_$r.log 2>&1 || { tail -5 $O/r6t24_base_$r.log; exit 1; }
  show $O/r6t24_base_$r.log base
  KUNGFU_DEV_KNOBS=1 KUNGFU_CONV_ROWS=1 timeout -k 10 300 python bench.py --steps 30 --warmup 8 --comm-probe 0 > $O/r6t24_rows_$r.log 2>&1 || { tail -5 $O/r6t24_rows_$r.log; exit 1; }
  show $O/r6t24_rows_$r.log rows
done
