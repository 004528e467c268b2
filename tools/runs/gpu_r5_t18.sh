#!/bin/bash
# r5 t18: conv epilogue via transposed product (8-byte LDS stores): GPU suite + ResNet / Inception bench + ResNet profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_wgrad_rows.py -x -q --timeout 600 --timeout-method thread -m gpu > $O/r5t18_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/r5t18_pytest.log | head -20; tail -1 $O/r5t18_pytest.log; [ $rc -eq 0 ] || exit $rc
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for M in resnet50 inception_v3; do
  timeout -k 10 300 python bench.py --model $M --steps 30 --warmup 6 > $O/r5t18_$M.log 2>&1 || { tail -5 $O/r5t18_$M.log; exit 1; }
  echo "$M: $(tail -1 $O/r5t18_$M.log | j)"
done
bash tools/gpu_prof.sh r5t18 resnet50 > $O/r5t18_prof.log 2>&1 && head -12 $O/r5t18_resnet50_summary.md
