#!/bin/bash
# The reference's other sync-scalability models on one MI355X: VGG16 and InceptionV3
# (224x224 synthetic, 256 images per GPU), bench.py + a rocprofv3 kernel-trace summary each.
# Usage (via gpurun): bash tools/gpu_models.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-models}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
for M in vgg16 inception_v3; do
  timeout -k 10 400 python bench.py --model $M --steps 20 --warmup 5 > "$OUT/${TAG}_${M}_bench.log" 2>&1 || exit $?
  tail -1 "$OUT/${TAG}_${M}_bench.log"
done
cd /tmp && export TMPDIR=/tmp
for M in vgg16 inception_v3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_${M}_prof" -o prof --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --model $M --steps 6 --warmup 3 > "$OUT/${TAG}_${M}_prof.log" 2>&1 || exit $?
  python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_${M}_prof/prof_kernel_trace.csv" --top 30 \
    > "$OUT/${TAG}_${M}_prof_summary.md" 2>&1
  head -22 "$OUT/${TAG}_${M}_prof_summary.md"
done
