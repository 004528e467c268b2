#!/bin/bash
# r6 t5: pipelined persistent 1x1 kernel: tests, per-op A/B, ResNet-50 A/B vs the no-pipe build, tile sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
SO=$(ls kungfu_amd/_hip*.so)
cp "$SO" /tmp/_hip_main.so
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_engine.py tests/test_gpu_gemm.py -x -q --timeout 300 --timeout-method thread \
  -k "conv or bottleneck or resnet or dgrad or bn_param or gemm" > $O/r6t5_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/r6t5_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
for V in main nopipe; do
  [ $V = main ] && cp /tmp/_hip_main.so "$SO" || cp alt/_hip_$V.so "$SO"
  timeout -k 10 300 python tools/bench_conv_epi.py --ops c1f,c3f > $O/r6t5_epi_$V.log 2>&1 || { tail -5 $O/r6t5_epi_$V.log; cp /tmp/_hip_main.so "$SO"; exit 1; }
  echo "$V: $(grep -v amdgpu $O/r6t5_epi_$V.log | tr '\n' ';')"
done
cp /tmp/_hip_main.so "$SO"
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for i in 1 2; do
  for V in main nopipe; do
    [ $V = main ] && cp /tmp/_hip_main.so "$SO" || cp alt/_hip_$V.so "$SO"
    timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/r6t5_bench_${V}_$i.log 2>&1 || { tail -5 $O/r6t5_bench_${V}_$i.log; cp /tmp/_hip_main.so "$SO"; exit 1; }
    echo "bench $V $i: $(tail -1 $O/r6t5_bench_${V}_$i.log | j)"
  done
done
cp /tmp/_hip_main.so "$SO"
VARIANTS=0,1,10,11,12 timeout -k 10 300 python tools/bench_bert_gemm.py > $O/r6t5_bert_gemm.log 2>&1; grep -v amdgpu.ids $O/r6t5_bert_gemm.log
timeout -k 10 900 python tools/bench_conv_tiles.py > $O/r6t5_tiles.log 2>&1; rc=$?
grep -v amdgpu.ids $O/r6t5_tiles.log
exit $rc
