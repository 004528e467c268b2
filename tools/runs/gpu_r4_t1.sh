#!/bin/bash
# round-4 GPU checks: new tests (preflight, comm emulator, >2 GiB fallback, hierarchical bf16, graph capture,
# gemm_nt), gemm_nt vs hipBLASLt, wgrad 32-pixel-stage A/B, convergence tests, then the emulation sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_rccl.py \
  tests/test_gpu.py tests/test_gpu_engine.py -k "preflight or emulate or 2gib or hierarchical or self_launch or watchdog or graphed or dropout" > $O/r4t1_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" $O/r4t1_pytest.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "gemm_nt or linear_gemm" > $O/r4t1_gemm.log 2>&1
rc=$?; tail -3 $O/r4t1_gemm.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm_nt.py > $O/r4t1_gemm_bench.log 2>&1 || { tail -20 $O/r4t1_gemm_bench.log; exit 1; }
cat $O/r4t1_gemm_bench.log
for kb in 0 1; do
  KUNGFU_DEV_KNOBS=1 KUNGFU_WGRAD_KB32=$kb VARIANTS=7 timeout -k 10 300 python tools/bench_wgrad_1x1.py > $O/r4t1_wgrad_kb$kb.log 2>&1 || { tail -20 $O/r4t1_wgrad_kb$kb.log; exit 1; }
  echo "== wgrad KB32=$kb"; cat $O/r4t1_wgrad_kb$kb.log
done
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_convergence.py > $O/r4t1_conv.log 2>&1
grep -E "acc|last-|stock|engine|passed|failed" $O/r4t1_conv.log | tail -12
bash tools/runs/gpu_r4_emu.sh
