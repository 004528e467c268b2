#!/bin/bash
# fused add+LayerNorm: numerics, BERT bench (+GNS) and kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2f}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -m gpu -k "layernorm or bert" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > "$OUT/${TAG}_bert.log" 2>&1 || { tail -30 "$OUT/${TAG}_bert.log"; exit 1; }
tail -1 "$OUT/${TAG}_bert.log" | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_bprof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model bert_base --optimizer gns --steps 6 --warmup 3 > "$OUT/${TAG}_bprof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_bprof/prof_kernel_trace.csv" --marker adam --top 24 > "$OUT/${TAG}_bprof_summary.md" 2>&1
head -34 "$OUT/${TAG}_bprof_summary.md"
