#!/bin/bash
# r5 t31: side-stream linear weight gradients (now default) under the multi-rank / elastic / graphed BERT tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_rccl.py tests/test_gpu_engine.py tests/test_gpu_convergence.py tests/test_gpu_gemm.py -k "bert or linear or gns or elastic" > $O/r5t31_pytest.log 2>&1
rc=$?; tail -1 $O/r5t31_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/r5t31_pytest.log | head -20; exit $rc; }
