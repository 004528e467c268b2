#!/bin/bash
# BN apply passes with non-temporal loads/stores (KUNGFU_BN_NT bit 0 loads, bit 1 stores):
# streaming micro-benchmark + ResNet-50 bench A/B.
set -o pipefail
export KUNGFU_DEV_KNOBS=1  # A/B of developer knobs (kungfu_amd/knobs.py)
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
hipcc -O3 --offload-arch=gfx950 tools/stream_bw.hip -o /tmp/stream_bw || exit 1
timeout -k 10 120 /tmp/stream_bw > "$OUT/r3f_stream_bw.txt" 2>&1 || exit $?
cat "$OUT/r3f_stream_bw.txt"
for nt in 0 3 1 2 0; do
  KUNGFU_BN_NT=$nt timeout -k 10 300 python bench.py --steps 30 --warmup 8 > "$OUT/r3f_bench_nt$nt.log" 2>&1 || exit $?
  echo "nt=$nt $(tail -1 $OUT/r3f_bench_nt$nt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
