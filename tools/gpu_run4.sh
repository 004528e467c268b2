#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 600 python -m pytest tests/test_gpu.py -q > gpurun_out/r4_pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_conv1x1.py > gpurun_out/r4_conv1x1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench.log 2>&1 || exit $?
