#!/bin/bash
# attention backward with 8 waves per workgroup: tests + A/B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu.py tests/test_gpu_engine.py -k "attention or attn or bert" > $O/r4t15_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/r4t15_pytest.log | head -30; [ $rc -eq 0 ] || exit $rc
for W in 8 4 8 4; do
KUNGFU_DEV_KNOBS=1 KUNGFU_ATTN_BWD_WAVES=$W timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t15_bert_w$W.log 2>&1 || { tail -20 $O/r4t15_bert_w$W.log; exit 1; }
echo "bert attn-bwd waves=$W $(tail -1 $O/r4t15_bert_w$W.log | j)"
done
