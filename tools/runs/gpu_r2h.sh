#!/bin/bash
# pipelined persistent conv kernel: numerics vs the reference kernel, then the 1x1 shape sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2h}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "pipe_kernel or persistent" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
MODES=st,,ab timeout -k 10 400 python tools/bench_conv1x1_variants.py > "$OUT/${TAG}_c1.log" 2>&1 || { tail -20 "$OUT/${TAG}_c1.log"; exit 1; }
cat "$OUT/${TAG}_c1.log"
