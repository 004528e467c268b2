#!/bin/bash
# r5 t5: segmented capture (relaxed mode), Inception deterministic capture test, emulated eager vs
# captured, host cost from an idle GPU, VGG per-layer NaN hunt (old vs new bias backward)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py::test_segmented_capture_with_emulated_comm_matches_eager \
  tests/test_gpu_engine.py::test_graphed_inception_v3_step_matches_eager \
  tests/test_gpu_rccl.py::test_bench_two_ranks_whole_step_graph \
  tests/test_gpu_rccl.py::test_bench_two_ranks_single_graph_layout > $O/r5t5_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|^eager|^graph|Error" $O/r5t5_pytest.log | head -40; tail -1 $O/r5t5_pytest.log
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); v=d["verify"]; print(d["value"], d["ms_per_step"], d["config"]["hip_graph"], v.get("exposed_comm_ms"), d["config"]["final_loss"])'; }
for rep in 1 2; do for cfg in "0 1" "1 1" "1 0"; do set -- $cfg
  KUNGFU_GRAPH_SEGMENTED=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 6 --emulate-comm 8 --emulate-ctas 16 --graph $1 > $O/r5t5_emu_$1$2_$rep.log 2>&1 || { tail -5 $O/r5t5_emu_$1$2_$rep.log; exit 1; }
  echo "emu8 graph=$1 seg=$2 rep=$rep $(tail -1 $O/r5t5_emu_$1$2_$rep.log | j)"
done; done
for M in resnet50 inception_v3; do
  timeout -k 10 300 python tools/diag/cpu_overhead.py $M > $O/r5t5_cpu_$M.log 2>&1 && grep host $O/r5t5_cpu_$M.log
done
# NaN hunt: VGG-16 per-layer path captured at batch 256 (the r4 failure), round-4 bias backward vs round-5
cp kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so /tmp/_hip_new.so
for v in old new; do
  [ $v = old ] && cp gpurun_extra/oldbias/_hip.cpython-310-x86_64-linux-gnu.so kungfu_amd/
  [ $v = new ] && cp /tmp/_hip_new.so kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so
  for i in 1 2 3 4 5 6; do
    KUNGFU_DEV_KNOBS=1 KUNGFU_VGG_FUSED=0 timeout -k 10 200 python bench.py --model vgg16 --graph 1 --steps 20 --warmup 5 > $O/r5t5_vgg_${v}_$i.log 2>&1 || { tail -3 $O/r5t5_vgg_${v}_$i.log; exit 1; }
    echo "vgg per-layer captured $v $i: $(tail -1 $O/r5t5_vgg_${v}_$i.log | j)"
  done
done
