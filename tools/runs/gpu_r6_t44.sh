#!/bin/bash
# r6 t44: VGG-16 with the row-image weight gradient on every 3x3 (round-6 plan) vs round 5; wgrad tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wgrad_rows.py tests/test_gpu.py -k "wgrad or vgg" > $O/r6t44_test.log 2>&1; rc=$?
tail -2 $O/r6t44_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/r6t44_test.log | head; exit $rc; }
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2; do
  for m in 1 2; do
    KUNGFU_DEV_KNOBS=1 KUNGFU_WGRAD_PLAN=$m timeout -k 10 300 python bench.py --model vgg16 --steps 15 --warmup 5 --comm-probe 0 > $O/r6t44_vgg_m${m}_$r.log 2>&1 || { tail -5 $O/r6t44_vgg_m${m}_$r.log; exit 1; }
    show $O/r6t44_vgg_m${m}_$r.log vgg16_plan$m
  done
done
