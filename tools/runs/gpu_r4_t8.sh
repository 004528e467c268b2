#!/bin/bash
# graph-default bench checks: multi-rank capture (colocated RCCL + host-plane fallback), graphed engine tests,
# default benches of the three conv models, configs 3/4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_engine.py \
  -k "self_launch or whole_step_graph or graphed" > $O/r4t8_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E |capture" $O/r4t8_pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"), d["config"]["comm"].get("comm_plane"))'; }
for M in resnet50 inception_v3 vgg16; do
  timeout -k 10 300 python bench.py --model $M --steps 30 --warmup 6 > $O/r4t8_$M.log 2>&1 || { tail -20 $O/r4t8_$M.log; exit 1; }
  echo "$M $(tail -1 $O/r4t8_$M.log | j)"
done
for o in sma pair; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 6 --optimizer $o > $O/r4t8_$o.log 2>&1 || { tail -20 $O/r4t8_$o.log; exit 1; }
  echo "$o $(tail -1 $O/r4t8_$o.log | j)"
done
timeout -k 10 300 python bench.py --steps 30 --warmup 6 --graph 0 > $O/r4t8_resnet50_eager.log 2>&1 && echo "resnet50 eager $(tail -1 $O/r4t8_resnet50_eager.log | j)"
