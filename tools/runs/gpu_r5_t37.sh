#!/bin/bash
# r5 t37: current-default BERT-base + GNS profile (hipBLASLt share) + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r5t37_bert.log 2>&1 || { tail -5 $O/r5t37_bert.log; exit 1; }
echo "bert: $(tail -1 $O/r5t37_bert.log | j)"
bash tools/gpu_prof.sh r5t37 bert_base > $O/r5t37_prof.log 2>&1 && head -24 $O/r5t37_bert_base_summary.md
python3 - <<'PY'
import re
rows = [l for l in open("gpurun_out/r5t37_bert_base_shapes.md") if l.startswith("| ") and "`" in l]
tot = sum(float(l.split("|")[1]) for l in rows)
blas = sum(float(l.split("|")[1]) for l in rows if "Cijk" in l)
print("kernel us/step %.1f, hipBLASLt %.1f (%.1f %%)" % (tot, blas, 100 * blas / tot))
PY
