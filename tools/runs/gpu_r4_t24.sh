#!/bin/bash
# 4-wave NT GEMM (128 x 128 per wave, asm MFMAs on AGPR accumulators): tests, then timings vs hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "gemm_nt" > $O/r4t24_pytest.log 2>&1
rc=$?; grep -E "FAILED|^E " $O/r4t24_pytest.log | head -20; tail -1 $O/r4t24_pytest.log; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=$PWD timeout -k 10 300 python tools/bench_gemm_nt.py > $O/r4t24_gemm_bench.log 2>&1; rc=$?; grep -v amdgpu.ids $O/r4t24_gemm_bench.log | cut -c1-330; exit $rc
