#!/bin/bash
# BERT-base + GNS: rocprofv3 kernel trace, eager vs whole-step capture (same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for G in 0 1; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/r4t32_g${G}_prof" -o prof --output-format csv -- \
    python3 "$R/bench.py" --model bert_base --optimizer gns --graph $G --steps 6 --warmup 3 > "$OUT/r4t32_g${G}_prof.log" 2>&1 || exit $?
  python3 "$R/tools/prof_summary.py" "$OUT/r4t32_g${G}_prof/prof_kernel_trace.csv" --top 40 --marker adam > "$OUT/r4t32_bert_g${G}_summary.md" 2>&1
  head -20 "$OUT/r4t32_bert_g${G}_summary.md"
done
