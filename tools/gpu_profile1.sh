#!/bin/bash
# Warm the MIOpen find-db, then profile a ResNet-50 autocast/channels_last step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/miopen_db gpurun_out/miopen_cache gpurun_out/prof1
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/miopen_cache
timeout -k 10 420 python tools/probe_resnet.py --variants autocast_cl --steps 10 --warmup 3 > gpurun_out/p2_warm.log 2>&1 || exit $?
timeout -k 10 200 python tools/probe_resnet.py --variants autocast_cl --steps 10 --warmup 3 > gpurun_out/p2_warm2.log 2>&1 || exit $?
timeout -k 10 200 python tools/probe_resnet.py --variants autocast_cl --steps 10 --warmup 3 --benchmark 0 > gpurun_out/p2_nobench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_resnet.py --variants autocast_cl --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/p2_prof.log 2>&1
