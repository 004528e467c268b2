#!/bin/bash
# persistent statistics epilogue: numerics (new + fused block tests), 1x1 sweep, ResNet-50 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2g}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "persistent or bottleneck or fused_block or conv" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
timeout -k 10 300 python tools/bench_conv1x1_variants.py > "$OUT/${TAG}_c1.log" 2>&1 || exit 1
cut -c1-110 "$OUT/${TAG}_c1.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/${TAG}_r50.log" 2>&1 || exit 1
tail -1 "$OUT/${TAG}_r50.log" | cut -c1-250
