#!/bin/bash
# r5 t20: wgrad split partials through the cache hierarchy (plain stores / loads) vs non-temporal: ResNet + BERT profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wgrad_rows.py tests/test_gpu.py -k "wgrad" > $O/r5t20_pytest.log 2>&1
rc=$?; tail -1 $O/r5t20_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r5t20 resnet50 bert_base > $O/r5t20_prof.log 2>&1 || { tail -5 $O/r5t20_prof.log; exit 1; }
for M in resnet50 bert_base; do grep -E "wgrad|conv MFMA 1x1|gemm" $O/r5t20_${M}_summary.md | head -4; grep -E "wgrad_reduce|wgrad_dense" $O/r5t20_${M}_shapes.md | head -5; done
