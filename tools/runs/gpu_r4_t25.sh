#!/bin/bash
# BERT: MLM-head LayerNorm on HIP, wider colsum stage 2 (tests + bench + profile); 4 colocated RCCL ranks
# with whole-step capture; Inception-v3 profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"), d["config"].get("final_loss"), d.get("verify",{}).get("replicas_consistent"))'; }
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_convergence.py tests/test_gpu.py -k "inception_bn_concat or layernorm" > $O/r4t25_pytest.log 2>&1
rc=$?; grep -E "FAILED|^E " $O/r4t25_pytest.log | head -20; tail -1 $O/r4t25_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t25_bert$i.log 2>&1 || { tail -20 $O/r4t25_bert$i.log; exit 1; }
echo "bert $(tail -1 $O/r4t25_bert$i.log | j)"
done
KUNGFU_FORCE_DEVICE=0 KUNGFU_RCCL_COLOCATE=1 NCCL_SOCKET_IFNAME=lo timeout -k 10 300 python bench.py --gpus 4 --batch 8 --steps 4 --warmup 4 > $O/r4t25_4rank.log 2>&1 || { grep -v "socket.cpp\|amdgpu.ids" $O/r4t25_4rank.log | tail -30; exit 1; }
echo "4 ranks $(tail -1 $O/r4t25_4rank.log | j)"
for F in 1 0 1 0; do
KUNGFU_DEV_KNOBS=1 KUNGFU_BN_BATCH_FIN=$F timeout -k 10 300 python bench.py --model inception_v3 --steps 30 --warmup 6 > $O/r4t25_inc_f$F.log 2>&1 || { tail -20 $O/r4t25_inc_f$F.log; exit 1; }
echo "inception batch_fin=$F $(tail -1 $O/r4t25_inc_f$F.log | j)"
done
bash tools/gpu_prof.sh r4t25 bert_base inception_v3 | grep -E "kernel sum"
