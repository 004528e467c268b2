#!/bin/bash
# r6 t46: row-image 3x3 conv with VGG's epilogues and the wide-map variant 26: tests, timing, VGG-16 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_rows.py > $O/r6t46_test.log 2>&1; rc=$?
tail -2 $O/r6t46_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/r6t46_test.log | head; exit $rc; }
for v in -1 26; do timeout -k 10 200 python -u tools/bench_vgg_conv.py --shape 0 --variant $v --iters 10 2>&1 | grep "H="; done
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2; do
  for m in 0 1; do
    KUNGFU_DEV_KNOBS=1 KUNGFU_CONV_ROWS_WIDE=$m timeout -k 10 300 python bench.py --model vgg16 --steps 15 --warmup 5 --comm-probe 0 > $O/r6t46_vgg_w${m}_$r.log 2>&1 || { tail -5 $O/r6t46_vgg_w${m}_$r.log; exit 1; }
    show $O/r6t46_vgg_w${m}_$r.log vgg16_wide$m
  done
done
