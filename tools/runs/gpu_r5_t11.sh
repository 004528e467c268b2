#!/bin/bash
# r5 t11: 32-channel rows wgrad (variant 8): numerics + per-shape timing vs MIOpen / 64-tile rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wgrad_rows.py > $O/r5t11_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|Error" $O/r5t11_pytest.log | head -20; tail -1 $O/r5t11_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_inception_wgrad.py > $O/r5t11_wgrad.txt 2>&1; rc=$?; cat $O/r5t11_wgrad.txt | grep -v amdgpu.ids; exit $rc
