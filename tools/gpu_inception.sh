#!/bin/bash
# Inception-v3 on one MI355X: its GPU numerics test, bench.py, rocprofv3 kernel-trace summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-inc}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k inception > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
timeout -k 10 400 python bench.py --model inception_v3 --steps 20 --warmup 5 > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model inception_v3 --steps 6 --warmup 3 > "$OUT/${TAG}_prof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_prof/prof_kernel_trace.csv" --top 30 \
  > "$OUT/${TAG}_prof_summary.md" 2>&1
head -20 "$OUT/${TAG}_prof_summary.md"
