#!/bin/bash
# Weight gradients on a side stream (KUNGFU_WGRAD_STREAM): numerics test + ResNet-50 A/B.
set -o pipefail
export KUNGFU_DEV_KNOBS=1  # A/B of developer knobs (kungfu_amd/knobs.py)
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_engine.py -k side_stream > "$OUT/r3k_side_test.log" 2>&1
rc=$?; tail -3 "$OUT/r3k_side_test.log"; [ $rc -eq 0 ] || exit $rc
for m in 0 1 0 1; do
  KUNGFU_WGRAD_STREAM=$m timeout -k 10 300 python bench.py --steps 30 --warmup 8 > "$OUT/r3k_bench_$m.log" 2>&1 || exit $?
  echo "wgrad_stream=$m $(tail -1 $OUT/r3k_bench_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
