#!/bin/bash
# 2-rank colocated RCCL bench: eager vs graph (segfault hunt), embedding kernel tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
export PYTHONFAULTHANDLER=1
: emb done

KUNGFU_FORCE_DEVICE=0 KUNGFU_RCCL_COLOCATE=1 NCCL_SOCKET_IFNAME=lo timeout -k 10 240 python bench.py --gpus 2 --steps 3 --warmup 2 --batch 16 --graph 0 > $O/r4t9_g0.log 2>&1
rc=$?; echo "graph0 rc=$rc"; tail -3 $O/r4t9_g0.log; [ $rc -eq 0 ] || exit $rc
KUNGFU_FORCE_DEVICE=0 KUNGFU_RCCL_COLOCATE=1 NCCL_SOCKET_IFNAME=lo timeout -k 10 240 python bench.py --gpus 2 --steps 3 --warmup 4 --batch 16 --graph 1 > $O/r4t9_g1.log 2>&1
rc=$?; echo "graph1 rc=$rc"; grep -v "socket.cpp\|amdgpu.ids" $O/r4t9_g1.log | tail -60
