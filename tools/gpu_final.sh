#!/bin/bash
# Round-end rehearsal on one MI355X: full GPU suite, smoke(), headline bench, Inception-v3 profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-final}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 240 --timeout-method thread -m gpu > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -2 "$OUT/${TAG}_pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || { tail -20 "$OUT/${TAG}_smoke.log"; exit 1; }
tail -1 "$OUT/${TAG}_smoke.log"
timeout -k 10 300 python bench.py > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_inc_prof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model inception_v3 --steps 6 --warmup 3 > "$OUT/${TAG}_inc_prof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_inc_prof/prof_kernel_trace.csv" --top 30 \
  > "$OUT/${TAG}_inc_prof_summary.md" 2>&1
head -20 "$OUT/${TAG}_inc_prof_summary.md"
