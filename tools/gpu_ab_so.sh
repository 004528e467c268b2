#!/bin/bash
# A/B of two builds of the HIP extension on the ResNet-50 bench (box-local swap of the .so):
#   tools/gpu_ab_so.sh <alt.so> <tag> [bench args...]
set -o pipefail
export KUNGFU_DEV_KNOBS=1  # A/B of developer knobs (kungfu_amd/knobs.py)
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
ALT=$1; TAG=$2; shift 2
BARGS=("$@")
SO=$(ls kungfu_amd/_hip*.so)
cp "$SO" /tmp/_hip_main.so
run() {  # $1 = label
  timeout -k 10 300 python bench.py --steps 30 --warmup 8 "${BARGS[@]}" > "$OUT/${TAG}_$1.log" 2>&1 || return $?
  echo "$1 $(tail -1 $OUT/${TAG}_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for i in 1 2; do
  cp /tmp/_hip_main.so "$SO" && run main$i || exit $?
  cp "$ALT" "$SO" && run alt$i || exit $?
done
cp /tmp/_hip_main.so "$SO"
