#!/bin/bash
# r6 t8: fused stem backward (stem_wgrad_bnp): tests, per-op timing, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread \
  > $O/r6t8_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $O/r6t8_pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_stem.py > $O/r6t8_stem.log 2>&1 || { tail -5 $O/r6t8_stem.log; exit 1; }
tail -6 $O/r6t8_stem.log
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for i in 1 2; do
  for V in 1 0; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 8 --stem-fused $V > $O/r6t8_s${V}_$i.log 2>&1 || { tail -5 $O/r6t8_s${V}_$i.log; exit 1; }
    echo "stem fused $V run $i: $(tail -1 $O/r6t8_s${V}_$i.log | j)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread \
  -k "resnet or bn_param" > $O/r6t8_engine.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/r6t8_engine.log | tail -5; exit $rc
