#!/bin/bash
# VGG-16 on one MI355X: bench.py + rocprofv3 kernel-trace summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-vgg}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model vgg16 --steps 6 --warmup 3 > "$OUT/${TAG}_prof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_prof/prof_kernel_trace.csv" --top 30 \
  > "$OUT/${TAG}_prof_summary.md" 2>&1
head -20 "$OUT/${TAG}_prof_summary.md"
