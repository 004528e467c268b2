#!/bin/bash
# r5 t8: after the knob retirement -- the touched GPU tests, a current-default BERT profile, and the
# Inception-v3 host profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_gemm.py tests/test_gpu_engine.py tests/test_gpu_embedding.py -k "not resnet50_engine_gradients and not memorises" > $O/r5t8_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/r5t8_pytest.log | head -20; tail -1 $O/r5t8_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r5t8 bert_base > $O/r5t8_prof.log 2>&1 || { tail -5 $O/r5t8_prof.log; exit 1; }
head -30 $O/r5t8_bert_base_summary.md
CPROFILE=1 timeout -k 10 300 python tools/diag/cpu_overhead.py inception_v3 > $O/r5t8_cprof_inception.log 2>&1 && grep host $O/r5t8_cprof_inception.log
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py -k "prebn" > $O/r5t8_prebn_test.log 2>&1; echo "prebn test rc=$? $(tail -1 $O/r5t8_prebn_test.log)"
timeout -k 10 300 python -u tools/bench_prebn.py > $O/r5t8_prebn.log 2>&1; echo "bench_prebn rc=$?"; cat $O/r5t8_prebn.log | grep -v "^/opt\|RCCL\|HIP v\|ROCm v\|Hostname\|Librccl"
