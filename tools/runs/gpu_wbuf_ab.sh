#!/bin/bash
# buffer-resource wgrad staging (alt .so) numerics + same-box A/B, after the round-end rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
bash tools/runs/gpu_final2.sh || exit 1
SO=$(ls kungfu_amd/_hip*.so)
cp "$SO" /tmp/_hip_main.so && cp alt/_hip_wbuf.so "$SO"
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_wgrad_rows.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "wgrad or bottleneck or resnet or inception or vgg or linear or bert" > $O/wbuf_alt_t.log 2>&1; rc=$?
cp /tmp/_hip_main.so "$SO"
echo "alt tests rc=$rc: $(tail -1 $O/wbuf_alt_t.log)"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/wbuf_alt_t.log | head -20; exit 1; }
bash tools/gpu_ab_so.sh alt/_hip_wbuf.so wbufab || exit 1
bash tools/gpu_ab_so.sh alt/_hip_wbuf.so wbufbert --model bert_base --optimizer gns || exit 1
