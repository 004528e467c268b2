#!/bin/bash
# r6 t30: the elastic BERT-GNS tests (both planes) after the wire-dtype fix, then the 224x256 tile run (t27)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 280 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread "tests/test_gpu_rccl.py::test_bench_elastic_bert_gns" > $O/r6t30_elastic.log 2>&1; rc=$?
echo "elastic rc=$rc"; grep -E "PASSED|FAILED|passed|failed" $O/r6t30_elastic.log | tail -4; [ $rc -eq 0 ] || exit $rc
bash tools/runs/gpu_r6_t27.sh
