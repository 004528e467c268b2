#!/bin/bash
# r5 t10: stem3 (Inception Conv2d_1a on MFMA) tests + Inception bench / profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py -k "stem3 or inception_stem" \
  tests/test_gpu_engine.py::test_graphed_inception_v3_step_matches_eager > $O/r5t10_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|Error" $O/r5t10_pytest.log | head -20; tail -1 $O/r5t10_pytest.log; [ $rc -eq 0 ] || exit $rc
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["hip_graph"], d["config"]["final_loss"])'; }
for S in 1 0; do
  KUNGFU_STEM=$S timeout -k 10 300 python bench.py --model inception_v3 --steps 30 --warmup 6 > $O/r5t10_inc_s$S.log 2>&1 || { tail -5 $O/r5t10_inc_s$S.log; exit 1; }
  echo "inception KUNGFU_STEM=$S: $(tail -1 $O/r5t10_inc_s$S.log | j)"
done
bash tools/gpu_prof.sh r5t10 inception_v3 > $O/r5t10_prof.log 2>&1 && head -24 $O/r5t10_inception_v3_summary.md
