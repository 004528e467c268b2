#!/bin/bash
# r6 t2: conv epilogue prefetch (PF=2 main, PF=0 / PF=1 alt): conv + engine tests, per-op bench, ResNet-50 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
SO=$(ls kungfu_amd/_hip*.so)
cp "$SO" /tmp/_hip_main.so
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread \
  -k "conv or bottleneck or resnet or dgrad or bn_param" > $O/r6t2_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/r6t2_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
grep "BN param grads" $O/r6t2_pytest.log
for V in main pf0 pf1; do
  [ $V = main ] && cp /tmp/_hip_main.so "$SO" || cp alt/_hip_$V.so "$SO"
  timeout -k 10 300 python tools/bench_conv_epi.py > $O/r6t2_epi_$V.log 2>&1 || { tail -5 $O/r6t2_epi_$V.log; cp /tmp/_hip_main.so "$SO"; exit 1; }
  echo "$V: $(tail -1 $O/r6t2_epi_$V.log)"
done
cp /tmp/_hip_main.so "$SO"
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for i in 1 2; do
  for V in main pf0 pf1; do
    [ $V = main ] && cp /tmp/_hip_main.so "$SO" || cp alt/_hip_$V.so "$SO"
    timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/r6t2_bench_${V}_$i.log 2>&1 || { tail -5 $O/r6t2_bench_${V}_$i.log; cp /tmp/_hip_main.so "$SO"; exit 1; }
    echo "bench $V $i: $(tail -1 $O/r6t2_bench_${V}_$i.log | j)"
  done
done
cp /tmp/_hip_main.so "$SO"
