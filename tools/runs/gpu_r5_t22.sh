#!/bin/bash
# r5 t22: quantisation-aware conv tile choice: conv tests + ResNet-50 bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_engine.py -k "conv or resnet or engine" > $O/r5t22_pytest.log 2>&1
rc=$?; tail -1 $O/r5t22_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED" $O/r5t22_pytest.log | head; exit $rc; }
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python bench.py > $O/r5t22_resnet50.log 2>&1 || { tail -5 $O/r5t22_resnet50.log; exit 1; }
echo "resnet50: $(tail -1 $O/r5t22_resnet50.log | j)"
bash tools/gpu_prof.sh r5t22 resnet50 > $O/r5t22_prof.log 2>&1 && head -10 $O/r5t22_resnet50_summary.md
