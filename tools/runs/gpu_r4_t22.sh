#!/bin/bash
# fused cross-entropy A/B, native pair prefetcher (tests + bench A/B), emulate test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"), d["config"].get("initial_loss"), d["config"].get("final_loss"))'; }
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu.py -k "pair or emulate" > $O/r4t22_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/r4t22_pytest.log | head -30; [ $rc -eq 0 ] || exit $rc
for X in 1 0 1 0; do
KUNGFU_DEV_KNOBS=1 KUNGFU_FUSED_XENT=$X timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t22_bert_x$X.log 2>&1 || { tail -20 $O/r4t22_bert_x$X.log; exit 1; }
echo "bert xent=$X $(tail -1 $O/r4t22_bert_x$X.log | j)"
done
for P in 1 0 1 0; do
KUNGFU_DEV_KNOBS=1 KUNGFU_PAIR_NATIVE=$P timeout -k 10 300 python bench.py --optimizer pair --steps 30 --warmup 6 > $O/r4t22_pair_n$P.log 2>&1 || { tail -20 $O/r4t22_pair_n$P.log; exit 1; }
echo "pair native=$P $(tail -1 $O/r4t22_pair_n$P.log | j) $(tail -1 $O/r4t22_pair_n$P.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d.get("verify",{}).get("pair"), d["config"].get("pair"))')"
done
