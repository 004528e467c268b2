#!/bin/bash
# r5 t33: FC1 + GELU on one gemm.hip launch: tests + BERT bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_embedding.py tests/test_gpu_engine.py -k "vocab or ragged or cross_entropy or tied or shadow or bert or gelu or linear" > $O/r5t33_pytest.log 2>&1
rc=$?; tail -1 $O/r5t33_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/r5t33_pytest.log | head -20; exit $rc; }
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r5t33_bert.log 2>&1 || { tail -5 $O/r5t33_bert.log; exit 1; }
echo "bert: $(tail -1 $O/r5t33_bert.log | j)"
bash tools/gpu_prof.sh r5t33 bert_base > $O/r5t33_prof.log 2>&1 && head -24 $O/r5t33_bert_base_summary.md && grep -E "Cijk|gemm_nt_kernel|Gelu" $O/r5t33_bert_base_shapes.md | head -12
