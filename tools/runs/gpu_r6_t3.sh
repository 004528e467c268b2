#!/bin/bash
# r6 t3: tile sweep of the conv ops with their epilogues, wgrad variant sweep (main .so = PF=2; pf0 alt)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
SO=$(ls kungfu_amd/_hip*.so)
cp "$SO" /tmp/_hip_main.so && cp alt/_hip_pf0.so "$SO"
timeout -k 10 600 python tools/bench_conv_tiles.py > $O/r6t3_tiles.log 2>&1; rc=$?
cat $O/r6t3_tiles.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || { cp /tmp/_hip_main.so "$SO"; exit $rc; }
timeout -k 10 300 python tools/bench_wgrad_1x1.py > $O/r6t3_wgrad.log 2>&1; rc=$?
cp /tmp/_hip_main.so "$SO"
cat $O/r6t3_wgrad.log | grep -v amdgpu.ids
exit $rc
