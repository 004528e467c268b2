#!/bin/bash
# r5 t27: vocab head on gemm_nt_ld (default "ours") tests + where the BERT step's small torch ops come from
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_embedding.py tests/test_gpu_engine.py -k "vocab or ragged or cross_entropy or tied or shadow or bert" > $O/r5t27_pytest.log 2>&1
rc=$?; tail -1 $O/r5t27_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/r5t27_pytest.log | head -20; exit $rc; }
timeout -k 10 400 python -u tools/diag/bert_small_ops.py > $O/r5t27_small_ops.log 2>&1; rc=$?
grep -v amdgpu.ids $O/r5t27_small_ops.log; [ $rc -eq 0 ] || exit $rc
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r5t27_bert.log 2>&1 || { tail -5 $O/r5t27_bert.log; exit 1; }
echo "bert: $(tail -1 $O/r5t27_bert.log | j)"
