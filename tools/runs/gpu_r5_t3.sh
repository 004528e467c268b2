#!/bin/bash
# r5 t3: capture tests, chaos, emulated 8-rank eager vs captured (corrected traffic, N-rank layout)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py::test_graphed_vgg16_per_layer_step_matches_eager \
  tests/test_gpu_engine.py::test_graphed_inception_v3_step_matches_eager > $O/r5t3_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|^eager|^graph|Error" $O/r5t3_pytest.log | head -30; tail -1 $O/r5t3_pytest.log
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); v=d["verify"]; print(d["value"], d["ms_per_step"], d["config"]["hip_graph"], v.get("comm_per_bucket_ms"), v.get("exposed_comm_ms"))'; }
for rep in 1 2; do for g in 0 1; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 6 --emulate-comm 8 --emulate-ctas 16 --graph $g > $O/r5t3_emu_g${g}_$rep.log 2>&1 || { tail -5 $O/r5t3_emu_g${g}_$rep.log; exit 1; }
  echo "emu8 graph=$g rep=$rep $(tail -1 $O/r5t3_emu_g${g}_$rep.log | j)"
done; done
bash tools/runs/gpu_r5_chaos.sh
