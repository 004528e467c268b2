#!/bin/bash
# conv-family numerics, then ResNet-50 bench and a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-epi}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "${KSEL:-conv or bottleneck or resnet50 or vgg or global_avg}" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -60 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
for M in ${MODELS:-resnet50}; do
  timeout -k 10 300 python bench.py --model $M --steps 20 --warmup 5 > "$OUT/${TAG}_${M}.log" 2>&1 || { tail -20 "$OUT/${TAG}_${M}.log"; exit 1; }
  tail -1 "$OUT/${TAG}_${M}.log" | cut -c1-230
done
[ "${PROF:-1}" = 1 ] && bash tools/gpu_prof.sh ${TAG}p resnet50 > /dev/null
exit 0
