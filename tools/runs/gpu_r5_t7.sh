#!/bin/bash
# r5 t7: fast deterministic bias backward (VGG per-layer timing + capture test), 8 colocated ranks,
# elastic BERT 4 -> 8, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 1500 python -u -m pytest -v -s --timeout 900 --timeout-method thread -m gpu \
  "tests/test_gpu.py::test_bias_act_matches_torch" \
  tests/test_gpu_engine.py::test_graphed_vgg16_per_layer_step_matches_eager \
  tests/test_gpu_rccl.py::test_bench_eight_colocated_ranks \
  tests/test_gpu_rccl.py::test_bench_elastic_bert_gns_four_to_eight_ranks > $O/r5t7_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|Error" $O/r5t7_pytest.log | head -30; tail -1 $O/r5t7_pytest.log
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); v=d["verify"]; print(d["value"], d["ms_per_step"], d["config"]["hip_graph"], d["config"]["final_loss"])'; }
for i in 1 2; do
  KUNGFU_DEV_KNOBS=1 KUNGFU_VGG_FUSED=0 timeout -k 10 200 python bench.py --model vgg16 --graph 1 --steps 20 --warmup 5 > $O/r5t7_vgg_$i.log 2>&1
  echo "vgg per-layer captured $i rc=$?: $(tail -1 $O/r5t7_vgg_$i.log | j)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r5t7_bench.log 2>&1 && echo "resnet50 default: $(tail -1 $O/r5t7_bench.log | j)"
