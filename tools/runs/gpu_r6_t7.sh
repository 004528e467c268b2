#!/bin/bash
# r6 t7: direct f32 conv wgrad into the flat slots: engine tests + bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "resnet or bottleneck or bn_param or side_stream or engine" > $O/r6t7_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/r6t7_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for i in 1 2; do
  for V in 1 0; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 8 --conv-wgrad-direct $V > $O/r6t7_d${V}_$i.log 2>&1 || { tail -5 $O/r6t7_d${V}_$i.log; exit 1; }
    echo "direct $V run $i: $(tail -1 $O/r6t7_d${V}_$i.log | j)"
  done
done
