#!/bin/bash
# r6 t50: BERT-base + GNS with the side stream (linear weight gradients) restricted to every 2nd / 4th CU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
A="--model bert_base --optimizer gns --steps 30 --warmup 8 --comm-probe 0"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/r6t50_all_$r.log 2>&1 || { tail -5 $O/r6t50_all_$r.log; exit 1; }; show $O/r6t50_all_$r.log side_all_cus
  for e in 2 4; do
    timeout -k 10 300 python tools/bench_switch.py kungfu_amd.parallel.mixed:_SIDE_CU_EVERY=$e -- $A > $O/r6t50_e${e}_$r.log 2>&1 || { tail -5 $O/r6t50_e${e}_$r.log; exit 1; }
    show $O/r6t50_e${e}_$r.log side_every$e
  done
done
