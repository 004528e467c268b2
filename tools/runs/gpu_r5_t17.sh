#!/bin/bash
# r5 t17: write/read bandwidth ceilings; monitor-reduction tests; BERT bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 5 120 ./tools/write_bw_bin > $O/r5_write_bw.txt 2>&1; cat $O/r5_write_bw.txt
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests -k "sumsq or gns or variance or noise or monitor or attention or attn" > $O/r5t17_pytest.log 2>&1
rc=$?; tail -1 $O/r5t17_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/r5t17_pytest.log | head; exit $rc; }
timeout -k 10 120 python3 tools/bench_attention.py > $O/r5t17_attn.txt 2>&1 && grep -v amdgpu $O/r5t17_attn.txt
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r5t17_bert.log 2>&1 || { tail -5 $O/r5t17_bert.log; exit 1; }
tail -1 $O/r5t17_bert.log | cut -c1-200
bash tools/gpu_prof.sh r5t17 bert_base > $O/r5t17_prof.log 2>&1 && head -24 $O/r5t17_bert_base_summary.md
