#!/bin/bash
# bench.py + rocprofv3 kernel-trace summary.  Usage: bash tools/gpu_prof.sh TAG [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 300 python bench.py --steps 30 --warmup 5 "$@" > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench.log" | cut -c1-260
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 3 "$@" > "$OUT/${TAG}_prof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_prof/prof_kernel_trace.csv" --top 40 \
  > "$OUT/${TAG}_prof_summary.md" 2>&1
head -20 "$OUT/${TAG}_prof_summary.md"
