#!/bin/bash
# r5 t14: row-image wgrad auto variant in Inception-v3: tests + bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wgrad_rows.py \
  tests/test_gpu_engine.py::test_graphed_inception_v3_step_matches_eager > $O/r5t14_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|Error" $O/r5t14_pytest.log | head -20; tail -1 $O/r5t14_pytest.log; [ $rc -eq 0 ] || exit $rc
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["hip_graph"], d["config"]["final_loss"])'; }
timeout -k 10 300 python bench.py --model inception_v3 --steps 30 --warmup 6 > $O/r5t14_inc.log 2>&1 || { tail -5 $O/r5t14_inc.log; exit 1; }
echo "inception: $(tail -1 $O/r5t14_inc.log | j)"
bash tools/gpu_prof.sh r5t14 inception_v3 > $O/r5t14_prof.log 2>&1 && head -24 $O/r5t14_inception_v3_summary.md && { grep -c "igemm\|MIOpen\|miopen" $O/r5t14_inception_v3_shapes.md || true; }
