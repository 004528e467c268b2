#!/bin/bash
# r6 t47: BERT-base + GNS: FC2 data gradient + GELU backward fused in gemm.hip (default) vs hipBLASLt + gelu_bwd_colsum
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_switch.py kungfu_amd.ops.linear:_GELU_GEMM=False -- --model bert_base --optimizer gns --steps 30 --warmup 8 --comm-probe 0 > $O/r6t47_unfused_$r.log 2>&1 || { tail -5 $O/r6t47_unfused_$r.log; exit 1; }
  show $O/r6t47_unfused_$r.log unfused
  timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 8 --comm-probe 0 > $O/r6t47_fused_$r.log 2>&1 || { tail -5 $O/r6t47_fused_$r.log; exit 1; }
  show $O/r6t47_fused_$r.log fused
done
