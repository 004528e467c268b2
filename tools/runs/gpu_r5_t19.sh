#!/bin/bash
# r5 t19: persistent attention backward (register prefetch): attention tests + bench + BERT bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests -k "attention or attn or bert" > $O/r5t19_pytest.log 2>&1
rc=$?; tail -1 $O/r5t19_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/r5t19_pytest.log | head; exit $rc; }
timeout -k 10 120 python3 tools/bench_attention.py > $O/r5t19_attn.txt 2>&1 && grep -v amdgpu $O/r5t19_attn.txt
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r5t19_bert.log 2>&1 || { tail -5 $O/r5t19_bert.log; exit 1; }
tail -1 $O/r5t19_bert.log | cut -c1-200
