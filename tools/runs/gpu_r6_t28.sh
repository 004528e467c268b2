#!/bin/bash
# r6 t28: the ResNet convergence test with and without the row-image 3x3 kernel; the elastic BERT test alone
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for r in 1 0; do
  KUNGFU_DEV_KNOBS=1 KUNGFU_CONV_ROWS=$r timeout -k 10 400 python -u -m pytest -x -q -s --timeout 380 --timeout-method thread \
    tests/test_gpu_convergence.py -k resnet50_engine_learns > $O/r6t28_conv_rows$r.log 2>&1; echo "rows=$r rc=$?"
  grep -E "seed|passed|failed|assert" $O/r6t28_conv_rows$r.log | head -12
done
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread "tests/test_gpu_rccl.py::test_bench_elastic_bert_gns" > $O/r6t28_elastic.log 2>&1; echo "elastic rc=$?"
tail -5 $O/r6t28_elastic.log
