#!/bin/bash
# One GPU round-trip: GPU tests (optionally filtered), a bench run and a
# rocprofv3 kernel-trace of a short bench.  Usage (on the box, via gpurun):
#   bash tools/gpu_check.sh <tag> [pytest -k expr] [extra bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
KEXPR=${2:-}
shift 2 2>/dev/null
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -m pytest tests/test_gpu.py -q -k "$KEXPR" > "$OUT/${TAG}_pytest.log" 2>&1
else
  timeout -k 10 600 python -m pytest tests/test_gpu.py -q > "$OUT/${TAG}_pytest.log" 2>&1
fi
rc=$?
tail -3 "$OUT/${TAG}_pytest.log"
# a pytest failure still lets us bench; a timeout/crash does not
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 "$@" > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 3 "$@" > "$OUT/${TAG}_prof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_prof/prof_kernel_trace.csv" --top 40 \
  > "$OUT/${TAG}_prof_summary.md" 2>&1
head -20 "$OUT/${TAG}_prof_summary.md"
