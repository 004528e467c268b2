#!/bin/bash
# BN finalize load order (main .so) checks + buffer-resource conv staging (alt .so) numerics and A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
SO=$(ls kungfu_amd/_hip*.so)
K="bn or bottleneck or finalize or conv or resnet or inception or vgg or gemm or stem"
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "$K" > $O/buf_main_t.log 2>&1 || { tail -30 $O/buf_main_t.log; exit 1; }
echo "main tests: $(tail -1 $O/buf_main_t.log)"
cp "$SO" /tmp/_hip_main.so && cp alt/_hip_buf.so "$SO"
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "$K" > $O/buf_alt_t.log 2>&1; rc=$?
cp /tmp/_hip_main.so "$SO"
echo "alt tests rc=$rc: $(tail -1 $O/buf_alt_t.log)"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/buf_alt_t.log | head -20; exit 1; }
bash tools/gpu_ab_so.sh alt/_hip_buf.so bufab || exit 1
bash tools/gpu_prof.sh r3fin resnet50 | grep -E "finalize|kernel sum|wall"
