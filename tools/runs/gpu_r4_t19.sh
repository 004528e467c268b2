#!/bin/bash
# multi-rank capture default: rccl tests, graphed engine tests, default benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
timeout -k 10 900 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_engine.py -k "self_launch or whole_step_graph or graph_disabled or hipgraph or cta_budget or graphed or ssgd_matches" > $O/r4t19_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/r4t19_pytest.log | head -30; [ $rc -eq 0 ] || exit $rc
for M in resnet50 inception_v3; do
  timeout -k 10 300 python bench.py --model $M --steps 30 --warmup 6 > $O/r4t19_$M.log 2>&1 || { tail -20 $O/r4t19_$M.log; exit 1; }
  echo "$M $(tail -1 $O/r4t19_$M.log | j)"
done
