#!/bin/bash
# r5 t4: segmented N-rank capture (emulated + 2 colocated ranks), VGG bias-backward A/B (old .so),
# capture reproducibility per model, emulated eager vs captured, host profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py::test_segmented_capture_with_emulated_comm_matches_eager \
  tests/test_gpu_engine.py::test_graphed_vgg16_per_layer_step_matches_eager \
  tests/test_gpu_rccl.py::test_bench_two_ranks_whole_step_graph \
  tests/test_gpu_rccl.py::test_bench_two_ranks_single_graph_layout \
  "tests/test_gpu.py::test_bias_act_matches_torch" > $O/r5t4_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|^eager|^graph|Error" $O/r5t4_pytest.log | head -40; tail -1 $O/r5t4_pytest.log
# A/B: the round-4 bias backward (hipMemsetAsync + f32 atomics) in an otherwise identical .so
cp kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so /tmp/_hip_new.so && cp gpurun_extra/oldbias/_hip.cpython-310-x86_64-linux-gnu.so kungfu_amd/
for i in 1 2; do
timeout -k 10 300 python -u -m pytest -v -s --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py::test_graphed_vgg16_per_layer_step_matches_eager > $O/r5t4_oldbias_$i.log 2>&1
echo "OLD bias_act run $i rc=$?"; grep -E "^eager|^graph|PASSED|FAILED|Assertion" $O/r5t4_oldbias_$i.log | head -8
done
cp /tmp/_hip_new.so kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so
for M in "inception_v3 16" "resnet50 16" "vgg16 16"; do
  timeout -k 10 300 python -u tools/diag/capture_repro.py $M > $O/r5t4_repro_${M% *}.log 2>&1 || { tail -5 $O/r5t4_repro_${M% *}.log; exit 1; }
  echo "== $M"; grep "vs eager1" $O/r5t4_repro_${M% *}.log
done
DETERMINISTIC=1 timeout -k 10 300 python -u tools/diag/capture_repro.py inception_v3 16 > $O/r5t4_repro_inc_det.log 2>&1 && { echo "== inception det"; grep "vs eager1" $O/r5t4_repro_inc_det.log; }
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); v=d["verify"]; print(d["value"], d["ms_per_step"], d["config"]["hip_graph"], v.get("exposed_comm_ms"))'; }
for rep in 1 2; do for cfg in "0 1" "1 1" "1 0"; do set -- $cfg
  KUNGFU_GRAPH_SEGMENTED=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 6 --emulate-comm 8 --emulate-ctas 16 --graph $1 > $O/r5t4_emu_$1$2_$rep.log 2>&1 || { tail -5 $O/r5t4_emu_$1$2_$rep.log; exit 1; }
  echo "emu8 graph=$1 seg=$2 rep=$rep $(tail -1 $O/r5t4_emu_$1$2_$rep.log | j)"
done; done
CPROFILE=1 timeout -k 10 300 python tools/diag/cpu_overhead.py resnet50 > $O/r5t4_cprof_resnet50.log 2>&1 && head -3 $O/r5t4_cprof_resnet50.log
