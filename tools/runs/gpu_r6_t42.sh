#!/bin/bash
# r6 t42: conv weight gradients straight into the flat f32 slot (fused_block._WGRAD_DIRECT): engine tests + ResNet-50 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_convergence.py -k "resnet or graph or engine" > $O/r6t42_test.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/r6t42_test.log | tail -30; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/r6t42_test.log | head; exit $rc; }
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2; do
  timeout -k 10 300 python tools/bench_switch.py kungfu_amd.ops.fused_block:_WGRAD_DIRECT=False -- --steps 30 --warmup 8 --comm-probe 0 > $O/r6t42_land_$r.log 2>&1 || { tail -5 $O/r6t42_land_$r.log; exit 1; }
  show $O/r6t42_land_$r.log landed
  timeout -k 10 300 python bench.py --steps 30 --warmup 8 --comm-probe 0 > $O/r6t42_direct_$r.log 2>&1 || { tail -5 $O/r6t42_direct_$r.log; exit 1; }
  show $O/r6t42_direct_$r.log direct
done
