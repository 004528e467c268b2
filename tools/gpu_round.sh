#!/bin/bash
# Round trip on one MI355X: GPU tests, conv3x3 kernel-vs-MIOpen bench, bench.py, rocprofv3 kernel trace.
# Usage (via gpurun): bash tools/gpu_round.sh <tag> [extra bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 700 python -u -m pytest tests/test_gpu.py -x -v --timeout 240 --timeout-method thread -m gpu > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?
tail -3 "$OUT/${TAG}_pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_conv3x3.py > "$OUT/${TAG}_conv3x3.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 "$@" > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench.log"
timeout -k 10 300 env KUNGFU_CONV3X3=0 python bench.py --steps 30 --warmup 5 "$@" > "$OUT/${TAG}_bench_noconv.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench_noconv.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 3 "$@" > "$OUT/${TAG}_prof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_prof/prof_kernel_trace.csv" --top 40 \
  > "$OUT/${TAG}_prof_summary.md" 2>&1
head -20 "$OUT/${TAG}_prof_summary.md"
