#!/bin/bash
# RCCL in a hipGraph with the collectives on the capture's origin stream and compute forked
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
export PYTHONFAULTHANDLER=1 KUNGFU_NATIVE_BACKTRACE=1 KUNGFU_FORCE_DEVICE=0 KUNGFU_RCCL_COLOCATE=1 NCCL_SOCKET_IFNAME=lo
export PYTHONPATH=$PWD
timeout -k 10 120 bin/kungfu-run -q -np 2 -H 127.0.0.1:2 -port-range 31100-31120 -port 31099 -allow-xgmi \
  python tests/workers/rccl_graph.py ofork,one > $O/r4t17_min.log 2>&1
rc=$?; echo "min rc=$rc"; grep -v "socket.cpp\|amdgpu.ids\|0x2d34a8" $O/r4t17_min.log | tail -30
