#!/bin/bash
# r6 t10: hardware bf16 rounding check, stem tests + per-op timing, stem fused A/B, the linear-gemm test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 60 ./tools/diag/cvt_check || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread \
  -k "stem or linear_gemm_path" > $O/r6t10_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $O/r6t10_pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_stem.py > $O/r6t10_stem.log 2>&1 || { tail -5 $O/r6t10_stem.log; exit 1; }
tail -6 $O/r6t10_stem.log
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for i in 1 2; do
  for V in 1 0; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 8 --stem-fused $V > $O/r6t10_s${V}_$i.log 2>&1 || { tail -5 $O/r6t10_s${V}_$i.log; exit 1; }
    echo "stem fused $V run $i: $(tail -1 $O/r6t10_s${V}_$i.log | j)"
  done
done
