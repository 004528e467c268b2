#!/bin/bash
# r6 t32: BERT-base + GNS with the step on a high-priority stream (side-stream weight gradients behind it)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
python -c "import torch;print('priority range',torch.cuda.Stream.priority_range())"
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2; do
  for p in 0 1; do
    timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 8 --comm-probe 0 --stream-priority $p > $O/r6t32_p${p}_$r.log 2>&1 || { tail -5 $O/r6t32_p${p}_$r.log; exit 1; }
    show $O/r6t32_p${p}_$r.log prio$p
  done
done
