#!/bin/bash
# Generalised fused BN (Inception channel counts) + bigger conv tiles: numerics, then
# Inception-v3 / VGG-16 / ResNet-50 benches and an Inception kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2c}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "pool or inception" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -60 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -2 "$OUT/${TAG}_pytest.log"
for M in inception_v3; do
  timeout -k 10 400 python bench.py --model $M --steps 20 --warmup 5 > "$OUT/${TAG}_$M.log" 2>&1 || { tail -30 "$OUT/${TAG}_$M.log"; exit 1; }
  tail -1 "$OUT/${TAG}_$M.log" | cut -c1-300
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_iprof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model inception_v3 --steps 6 --warmup 3 > "$OUT/${TAG}_iprof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_iprof/prof_kernel_trace.csv" --top 40 > "$OUT/${TAG}_iprof_summary.md" 2>&1
head -24 "$OUT/${TAG}_iprof_summary.md"
