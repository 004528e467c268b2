#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
for cfg in "--steps 6 --warmup 3" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --optimizer local" "--steps 20 --warmup 5 --overlap 0"; do
  echo "=== $cfg" >> gpurun_out/r3_bench.log
  timeout -k 10 200 python bench.py $cfg >> gpurun_out/r3_bench.log 2>&1 || exit $?
done
echo "=== prio0" >> gpurun_out/r3_bench.log
KUNGFU_COMM_STREAM_PRIORITY=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/r3_bench.log 2>&1 || exit $?
echo "=== probe torch" >> gpurun_out/r3_bench.log
timeout -k 10 200 python tools/probe_resnet.py --variants autocast_cl --steps 20 --warmup 5 --benchmark 0 >> gpurun_out/r3_bench.log 2>&1 || exit $?
