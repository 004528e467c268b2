#!/bin/bash
# BN apply grid cap (KUNGFU_BN_MAXGRID) x non-temporal mode (KUNGFU_BN_NT) on the ResNet-50 bench.
set -o pipefail
export KUNGFU_DEV_KNOBS=1  # A/B of developer knobs (kungfu_amd/knobs.py)
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
for cfg in "1 2048" "1 1024" "1 4096" "3 1024" "1 2048" "0 2048"; do
  set -- $cfg
  KUNGFU_BN_NT=$1 KUNGFU_BN_MAXGRID=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 8 > "$OUT/r3g_bench_$1_$2.log" 2>&1 || exit $?
  echo "nt=$1 grid=$2 $(tail -1 $OUT/r3g_bench_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
