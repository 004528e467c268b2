#!/bin/bash
# Conv A operand staged with non-temporal LDS-DMA loads (KUNGFU_CONV_NT_A 0/1/2), ResNet-50 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
for m in 0 1 2 0 1 2; do
  KUNGFU_CONV_NT_A=$m timeout -k 10 300 python bench.py --steps 30 --warmup 8 > "$OUT/r3h_bench_$m.log" 2>&1 || exit $?
  echo "conv_nt_a=$m $(tail -1 $OUT/r3h_bench_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
