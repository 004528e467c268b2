#!/bin/bash
# RCCL collective inside a hipGraph capture, 2 colocated ranks: minimal worker, then the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
export PYTHONFAULTHANDLER=1 KUNGFU_NATIVE_BACKTRACE=1 KUNGFU_FORCE_DEVICE=0 KUNGFU_RCCL_COLOCATE=1 NCCL_SOCKET_IFNAME=lo
export PYTHONPATH=$PWD NCCL_GRAPH_MIXING_SUPPORT=${MIX:-0}
timeout -k 10 120 bin/kungfu-run -q -np 2 -H 127.0.0.1:2 -port-range 31100-31120 -port 31099 -allow-xgmi \
  python tests/workers/rccl_graph.py > $O/r4t10_min.log 2>&1
rc=$?; echo "min rc=$rc"; grep -v "socket.cpp\|amdgpu.ids" $O/r4t10_min.log | tail -70; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --gpus 2 --steps 3 --warmup 4 --batch 16 --graph 1 > $O/r4t10_g1.log 2>&1
rc=$?; echo "graph1 rc=$rc"; grep -v "socket.cpp\|amdgpu.ids" $O/r4t10_g1.log | grep -v "^  File\|^Extension" | tail -60
