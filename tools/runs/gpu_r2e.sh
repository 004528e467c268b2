#!/bin/bash
# wgrad split heuristic: VGG wgrad sweep default column + VGG-16 / ResNet-50 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2e}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "wgrad or vgg" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
for M in vgg16 resnet50; do
  timeout -k 10 400 python bench.py --model $M --steps 20 --warmup 5 > "$OUT/${TAG}_$M.log" 2>&1 || { tail -30 "$OUT/${TAG}_$M.log"; exit 1; }
  tail -1 "$OUT/${TAG}_$M.log" | cut -c1-260
done
