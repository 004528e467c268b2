#!/bin/bash
# r6 t25: conv epilogue bf16 rounding on v_cvt_pk_bf16_f32 (alt build, KFK_CONV_HWCVT=1) vs integer rounding:
# isolated 3x3 / 1x1 shapes, then the ResNet-50 bench (box-local .so swap)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
SO=$(ls kungfu_amd/_hip*.so); cp "$SO" /tmp/_hip_main.so
for arm in main alt; do
  if [ $arm = alt ]; then cp tools/alt/_hip_alt.so "$SO"; else cp /tmp/_hip_main.so "$SO"; fi
  timeout -k 10 200 python tools/bench_conv3x3_s1.py -1 > $O/r6t25_k3_$arm.log 2>&1 || { cp /tmp/_hip_main.so "$SO"; tail -5 $O/r6t25_k3_$arm.log; exit 1; }
  echo "== $arm"; cat $O/r6t25_k3_$arm.log | grep H=
  VARIANTS=-1 MODES=st,ab timeout -k 10 200 python tools/bench_conv1x1_variants.py > $O/r6t25_k1_$arm.log 2>&1 || { cp /tmp/_hip_main.so "$SO"; tail -5 $O/r6t25_k1_$arm.log; exit 1; }
  cat $O/r6t25_k1_$arm.log | grep H=
done
cp /tmp/_hip_main.so "$SO"
bash tools/gpu_ab_so.sh tools/alt/_hip_alt.so r6t25 --comm-probe 0
