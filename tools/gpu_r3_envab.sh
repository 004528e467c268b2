#!/bin/bash
# A/B of one environment variable on a model bench (1 GPU):
#   tools/gpu_r3_envab.sh <VAR> <a> <b> <tag> [bench args...]
set -o pipefail
export KUNGFU_DEV_KNOBS=1  # A/B of developer knobs (kungfu_amd/knobs.py)
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
VAR=$1; A=$2; B=$3; TAG=$4; shift 4
for v in $A $B $A $B; do
  env "$VAR=$v" timeout -k 10 300 python bench.py --steps 30 --warmup 8 "$@" > "$OUT/${TAG}_$v.log" 2>&1 || exit $?
  echo "$VAR=$v $(tail -1 $OUT/${TAG}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
