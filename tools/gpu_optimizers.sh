#!/bin/bash
# Full GPU test suite + ResNet-50 throughput for every distributed optimizer on 1 GPU
# (configs 2-4 of BASELINE.json: S-SGD, SMA, pair averaging; AdaSGD).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > "$OUT/opt_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/opt_pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for o in ssgd sma pair ada; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --optimizer $o > "$OUT/opt_bench_$o.log" 2>&1 || exit $?
  echo "$o $(tail -1 $OUT/opt_bench_$o.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
