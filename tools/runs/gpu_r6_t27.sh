#!/bin/bash
# r6 t27: 224x256 conv tile (variant 8): tests, isolated 14x14 timings vs 256x256, ResNet-50 A/B (KUNGFU_CONV_T224)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_tiles.py tests/test_gpu_conv_rows.py > $O/r6t27_test.log 2>&1; rc=$?
tail -3 $O/r6t27_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/r6t27_test.log | head; exit $rc; }
VARIANTS=7,8 MODES=st,bc timeout -k 10 200 python tools/bench_conv1x1_variants.py > $O/r6t27_k1.log 2>&1 || { tail -5 $O/r6t27_k1.log; exit 1; }
grep "H=14\|H= 7" $O/r6t27_k1.log
SHAPES=2 timeout -k 10 200 python tools/bench_conv3x3_s1.py 7 8 > $O/r6t27_k3.log 2>&1 || { tail -5 $O/r6t27_k3.log; exit 1; }
cat $O/r6t27_k3.log | grep H=
show() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['ms_per_step'],d['value'],d['config']['final_loss'])" $1 $2; }
for r in 1 2; do
  KUNGFU_DEV_KNOBS=1 KUNGFU_CONV_T224=0 timeout -k 10 300 python bench.py --steps 30 --warmup 8 --comm-probe 0 > $O/r6t27_base_$r.log 2>&1 || { tail -5 $O/r6t27_base_$r.log; exit 1; }
  show $O/r6t27_base_$r.log t256
  timeout -k 10 300 python bench.py --steps 30 --warmup 8 --comm-probe 0 > $O/r6t27_t224_$r.log 2>&1 || { tail -5 $O/r6t27_t224_$r.log; exit 1; }
  show $O/r6t27_t224_$r.log t224
done
