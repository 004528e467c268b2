#!/bin/bash
# rocprofv3 kernel summaries of the ResNet-50 bench with the in-tree extension and with an
# alternative build of it (box-local .so swap): tools/gpu_prof_ab.sh <alt.so> <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
ALT=$1; TAG=$2
SO=$(ls kungfu_amd/_hip*.so)
cp "$SO" /tmp/_hip_main.so
bash tools/gpu_prof.sh ${TAG}main resnet50 > /dev/null || exit $?
cp "$ALT" "$SO" && bash tools/gpu_prof.sh ${TAG}alt resnet50 > /dev/null; rc=$?
cp /tmp/_hip_main.so "$SO"
head -20 "$OUT/${TAG}main_resnet50_summary.md"; head -20 "$OUT/${TAG}alt_resnet50_summary.md"
exit $rc
