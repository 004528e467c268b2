#!/bin/bash
# --emulate-comm sweep (VERDICT r3 #1c): CTAs per all-reduce x bucket size, ResNet-50 at N=1 with
# the local footprint of an 8-rank ring all-reduce on the comm stream.  Prints one line per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
TAG=${TAG:-r4emu}
MODEL=${MODEL:-resnet50}
BUSBW=${BUSBW:-350}
CTAS=${CTAS:-"4 8 16 32"}
BUCKETS=${BUCKETS:-"8 16 32 64"}
run() {  # name, extra args...
  local n=$1; shift
  timeout -k 10 200 python bench.py --model $MODEL --steps 20 --warmup 5 "$@" > $O/${TAG}_$n.log 2>&1 || { tail -5 $O/${TAG}_$n.log; return 1; }
  echo "$n $(tail -1 $O/${TAG}_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]["comm"]; e=c.get("emulated") or {}; print(d["value"], d["ms_per_step"], c["buckets"], c["bucket_mb"], e.get("modelled_comm_ms_total"), e.get("calls"))')"
}
run base || exit 1
for B in $BUCKETS; do
  for C in $CTAS; do
    KUNGFU_BUCKET_MB=$B run b${B}_c${C} --emulate-comm 8 --emulate-ctas $C --emulate-busbw $BUSBW || exit 1
  done
done
