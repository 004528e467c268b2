#!/bin/bash
# r5 t29: split-K decoder data gradient: vocab tests + BERT bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_embedding.py tests/test_gpu_engine.py -k "vocab or ragged or cross_entropy or tied or shadow or bert" > $O/r5t29_pytest.log 2>&1
rc=$?; tail -1 $O/r5t29_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/r5t29_pytest.log | head -20; exit $rc; }
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r5t29_bert.log 2>&1 || { tail -5 $O/r5t29_bert.log; exit 1; }
echo "bert: $(tail -1 $O/r5t29_bert.log | j)"
bash tools/gpu_prof.sh r5t29 bert_base > $O/r5t29_prof.log 2>&1 && head -24 $O/r5t29_bert_base_summary.md && grep -E "Cijk|xent|gemm_nt_kernel<256, 1>|reduce_kernel" $O/r5t29_bert_base_shapes.md | head -12
