#!/bin/bash
# r5 t6: segmented capture without empty segments; emulated eager vs captured for ResNet-50 and
# Inception-v3; VGG per-layer NaN hunt (old vs new bias backward)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py::test_segmented_capture_with_emulated_comm_matches_eager \
  tests/test_gpu_rccl.py::test_bench_two_ranks_whole_step_graph > $O/r5t6_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|Error" $O/r5t6_pytest.log | head -20; tail -1 $O/r5t6_pytest.log; [ $rc -eq 0 ] || exit $rc
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); v=d["verify"]; print(d["value"], d["ms_per_step"], d["config"]["hip_graph"], v.get("exposed_comm_ms"), d["config"]["final_loss"])'; }
for M in resnet50 inception_v3; do for rep in 1 2; do for g in 0 1; do
  timeout -k 10 300 python bench.py --model $M --steps 30 --warmup 6 --emulate-comm 8 --emulate-ctas 16 --graph $g > $O/r5t6_emu_${M}_$g$rep.log 2>&1 || { tail -5 $O/r5t6_emu_${M}_$g$rep.log; exit 1; }
  echo "$M emu8 graph=$g rep=$rep $(tail -1 $O/r5t6_emu_${M}_$g$rep.log | j)"
done; done; done
cp kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so /tmp/_hip_new.so
for v in new old; do
  [ $v = old ] && cp gpurun_extra/oldbias/_hip.cpython-310-x86_64-linux-gnu.so kungfu_amd/
  for i in 1 2 3 4 5 6; do
    KUNGFU_DEV_KNOBS=1 KUNGFU_VGG_FUSED=0 timeout -k 10 200 python bench.py --model vgg16 --graph 1 --steps 20 --warmup 5 > $O/r5t6_vgg_${v}_$i.log 2>&1
    rc=$?; [ $rc -eq 0 ] || [ $rc -eq 4 ] || { echo "vgg $v $i rc=$rc"; tail -3 $O/r5t6_vgg_${v}_$i.log; exit 1; }
    echo "vgg per-layer captured $v $i rc=$rc: $(tail -1 $O/r5t6_vgg_${v}_$i.log | j)"
  done
done
cp /tmp/_hip_new.so kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so
