#!/bin/bash
# Inception-v3 convolutions on the MFMA kernel: numerics, benches, kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-inc}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "conv_rect or basicconv or inception or conv_flip or sibling or bn_link or conv3x3 or persistent or channel_slice or fused_bn or bn_" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -60 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
for M in inception_v3 resnet50; do
  timeout -k 10 300 python bench.py --model $M --steps 20 --warmup 5 > "$OUT/${TAG}_${M}.log" 2>&1 || { tail -20 "$OUT/${TAG}_${M}.log"; exit 1; }
  tail -1 "$OUT/${TAG}_${M}.log" | cut -c1-200
done
bash tools/gpu_prof.sh ${TAG}p inception_v3 > /dev/null
