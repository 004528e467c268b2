#!/bin/bash
# round-4 GPU checks: new tests (preflight, comm emulator, >2 GiB fallback, hierarchical bf16, gemm_nt),
# the gemm_nt vs hipBLASLt bench, convergence tests, then the emulation sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_rccl.py \
  tests/test_gpu.py -k "preflight or emulate or 2gib or hierarchical or self_launch or watchdog" > $O/r4t1_pytest.log 2>&1 || { tail -60 $O/r4t1_pytest.log; exit 1; }
tail -3 $O/r4t1_pytest.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k gemm_nt > $O/r4t1_gemm.log 2>&1 || { tail -40 $O/r4t1_gemm.log; exit 1; }
tail -2 $O/r4t1_gemm.log
timeout -k 10 300 python tools/bench_gemm_nt.py > $O/r4t1_gemm_bench.log 2>&1 || { tail -20 $O/r4t1_gemm_bench.log; exit 1; }
cat $O/r4t1_gemm_bench.log
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_convergence.py > $O/r4t1_conv.log 2>&1
grep -E "acc|last-|stock|engine|passed|failed" $O/r4t1_conv.log | tail -12
bash tools/runs/gpu_r4_emu.sh
