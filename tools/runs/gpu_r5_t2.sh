#!/bin/bash
# r5 t2: new / changed GPU tests (numerics envelope, capture races, bias backward, preflight stall), then chaos
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py::test_graphed_vgg16_per_layer_step_matches_eager \
  tests/test_gpu_engine.py::test_graphed_inception_v3_step_matches_eager \
  tests/test_gpu_engine.py::test_resnet50_engine_gradients_within_stock_bf16_envelope \
  "tests/test_gpu.py::test_bias_act_matches_torch" \
  tests/test_gpu.py::test_comm_emulate_kernel_paces_and_keeps_bucket \
  tests/test_gpu_rccl.py::test_bench_preflight_stall_skips_ipc_on_every_rank \
  tests/test_gpu_rccl.py::test_bench_self_launch_two_ranks > $O/r5t2_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|^eager|^graph|worst" $O/r5t2_pytest.log | head -60; tail -1 $O/r5t2_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/gpu_r5_chaos.sh
