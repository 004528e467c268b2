#!/bin/bash
# embedding gradient kernel (run-length) tests + timing, BERT small-kernel origins, BERT bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_embedding.py > $O/r4t12_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/r4t12_pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/diag/bert_fills.py > $O/r4t12_fills.log 2>&1; rc=$?; cat $O/r4t12_fills.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t12_bert.log 2>&1 || { tail -20 $O/r4t12_bert.log; exit 1; }
echo "bert $(tail -1 $O/r4t12_bert.log | j)"
