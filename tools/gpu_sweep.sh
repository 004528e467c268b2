#!/bin/bash
# 1x1 conv tile sweep: VARIANTS / MODES from the environment
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-sweep}
mkdir -p "$OUT"
timeout -k 10 400 python tools/bench_conv1x1_variants.py > "$OUT/${TAG}.log" 2>&1 || { tail -20 "$OUT/${TAG}.log"; exit 1; }
cat "$OUT/${TAG}.log"
