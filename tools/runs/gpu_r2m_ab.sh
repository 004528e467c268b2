#!/bin/bash
# A/B of an environment switch on one box: numerics, then the ResNet-50 bench alternating
# AB_VAR=0 / AB_VAR=1 (two rounds each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-ab}
VAR=${AB_VAR:?AB_VAR}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "${KSEL:-conv or bottleneck or resnet50 or global_avg}" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -60 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
for r in 1 2; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 300 python bench.py --model ${MODEL:-resnet50} --steps 30 --warmup 5 > "$OUT/${TAG}_${v}_$r.log" 2>&1 || { tail -20 "$OUT/${TAG}_${v}_$r.log"; exit 1; }
    echo "$VAR=$v: $(tail -1 "$OUT/${TAG}_${v}_$r.log" | grep -o "\"value\": [0-9.]*")"
  done
done
