#!/bin/bash
# Round 2, first GPU pass: engine tests (RCCL 1-rank path, bf16 wire, elastic GPU), the GPU
# suite, default bench (forced comm) vs skip mode, and a kernel trace of the forced-comm step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2a}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu.py -x -v --timeout 240 --timeout-method thread -m gpu > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -2 "$OUT/${TAG}_pytest.log"
timeout -k 10 300 python bench.py > "$OUT/${TAG}_bench_comm.log" 2>&1 || { tail -20 "$OUT/${TAG}_bench_comm.log"; exit 1; }
tail -1 "$OUT/${TAG}_bench_comm.log"
timeout -k 10 300 python bench.py --force-comm 0 > "$OUT/${TAG}_bench_skip.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench_skip.log"
timeout -k 10 300 python bench.py --comm-dtype bf16 > "$OUT/${TAG}_bench_bf16.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench_bf16.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 3 > "$OUT/${TAG}_prof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_prof/prof_kernel_trace.csv" --top 40 \
  > "$OUT/${TAG}_prof_summary.md" 2>&1
python3 "$GRAFT_REPO_ROOT/tools/prof_overlap.py" "$OUT/${TAG}_prof/prof_kernel_trace.csv" \
  > "$OUT/${TAG}_prof_overlap.md" 2>&1
head -16 "$OUT/${TAG}_prof_summary.md"
cat "$OUT/${TAG}_prof_overlap.md"
