#!/bin/bash
# row-image 3x3 wgrad: numerics (every variant) + per-variant timing on ResNet/VGG shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2i}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "wgrad" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
timeout -k 10 400 python tools/bench_wgrad_rows.py > "$OUT/${TAG}_w.log" 2>&1 || { tail -20 "$OUT/${TAG}_w.log"; exit 1; }
cat "$OUT/${TAG}_w.log"
