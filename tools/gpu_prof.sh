#!/bin/bash
# rocprofv3 kernel trace of bench.py per model: category summary + per-launch-shape table
# Usage (via gpurun): bash tools/gpu_prof.sh <tag> [models...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-prof}; shift
MODELS=${@:-resnet50}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/kungfu_amd/tuning/miopen
cd /tmp && export TMPDIR=/tmp
for M in $MODELS; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_${M}_prof" -o prof --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --model $M $( [ "${M#bert}" != "$M" ] && echo --optimizer gns ) --steps 6 --warmup 3 \
    > "$OUT/${TAG}_${M}_prof.log" 2>&1 || exit $?
  MK=sgd; case $M in bert*) MK=adam;; esac
  python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_${M}_prof/prof_kernel_trace.csv" --top 40 --marker $MK \
    > "$OUT/${TAG}_${M}_summary.md" 2>&1
  python3 "$GRAFT_REPO_ROOT/tools/prof_shapes.py" "$OUT/${TAG}_${M}_prof/prof_kernel_trace.csv" --top 70 --marker $MK \
    > "$OUT/${TAG}_${M}_shapes.md" 2>&1
  head -24 "$OUT/${TAG}_${M}_summary.md"
done
