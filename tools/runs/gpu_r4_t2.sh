#!/bin/bash
# round-4: gemm_nt (pipelined, conflict-free swizzle) tests + bench, graph/dropout/linear tests, convergence with logs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "gemm_nt or linear_gemm" > $O/r4t2_gemm.log 2>&1
rc=$?; tail -3 $O/r4t2_gemm.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm_nt.py > $O/r4t2_gemm_bench.log 2>&1 || { tail -20 $O/r4t2_gemm_bench.log; exit 1; }
cat $O/r4t2_gemm_bench.log
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu.py -k "graphed or dropout" > $O/r4t2_graph.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/r4t2_graph.log | head -20; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/diag/grad_compare.py > $O/r4t2_gradcmp.log 2>&1; tail -60 $O/r4t2_gradcmp.log
