#!/bin/bash
# Conv A operand / wgrad operands staged with non-temporal LDS-DMA loads
# (KUNGFU_CONV_NT_A, KUNGFU_WGRAD_NT: 0 off, 1 read-once operands, 2 always), ResNet-50 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
for cfg in "0 0" "1 0" "2 0" "0 1" "0 2" "1 1" "0 0" "1 1"; do
  set -- $cfg
  KUNGFU_CONV_NT_A=$1 KUNGFU_WGRAD_NT=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 8 > "$OUT/r3h_bench_$1_$2.log" 2>&1 || exit $?
  echo "conv_nt_a=$1 wgrad_nt=$2 $(tail -1 $OUT/r3h_bench_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
