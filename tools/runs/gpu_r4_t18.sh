#!/bin/bash
# multi-rank whole-step capture (comm stream as capture origin): 2 colocated RCCL ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
export PYTHONFAULTHANDLER=1 KUNGFU_NATIVE_BACKTRACE=1 KUNGFU_FORCE_DEVICE=0 KUNGFU_RCCL_COLOCATE=1 NCCL_SOCKET_IFNAME=lo
KUNGFU_DEV_KNOBS=1 KUNGFU_GRAPH_MULTIRANK=1 timeout -k 10 240 python bench.py --gpus 2 --steps 4 --warmup 4 --batch 16 --graph 1 > $O/r4t18_g1.log 2>&1
rc=$?; echo "graph1 rc=$rc"; grep -v "socket.cpp\|amdgpu.ids\|0x2d34a8" $O/r4t18_g1.log | tail -5 | cut -c1-2500
