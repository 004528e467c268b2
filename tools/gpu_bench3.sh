#!/bin/bash
# full GPU suite, then ResNet-50 / VGG-16 / Inception-v3 benches (1 GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-b3}
SUITE=${SUITE:-1}
MODELS=${MODELS:-"resnet50 vgg16 inception_v3"}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
if [ "$SUITE" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
  tail -1 "$OUT/${TAG}_pytest.log"
fi
for M in $MODELS; do
  timeout -k 10 300 python bench.py --model $M --steps 20 --warmup 5 > "$OUT/${TAG}_${M}.log" 2>&1 || { tail -20 "$OUT/${TAG}_${M}.log"; exit 1; }
  tail -1 "$OUT/${TAG}_${M}.log" | cut -c1-260
done
