#!/bin/bash
# r5 t23: FC2 data gradient + GELU backward fused on gemm.hip: tests + BERT bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu.py tests/test_gpu_engine.py -k "gemm or gelu or bert or linear" > $O/r5t23_pytest.log 2>&1
rc=$?; tail -1 $O/r5t23_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/r5t23_pytest.log | head; exit $rc; }
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r5t23_bert.log 2>&1 || { tail -5 $O/r5t23_bert.log; exit 1; }
echo "bert: $(tail -1 $O/r5t23_bert.log | j)"
bash tools/gpu_prof.sh r5t23 bert_base > $O/r5t23_prof.log 2>&1 && head -14 $O/r5t23_bert_base_summary.md && grep -E "gemm_nt|gelu|Cijk" $O/r5t23_bert_base_shapes.md | head -8
