#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/gpu_sanity.py > gpurun_out/r1_sanity.log 2>&1 || exit $?
timeout -k 10 120 python tools/gpu_sanity_bn.py > gpurun_out/r1_sanity_bn.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fused-bn 0 > gpurun_out/r1_bench_nofuse.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fused-bn 1 > gpurun_out/r1_bench_fuse.log 2>&1 || exit $?
