#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof2
timeout -k 10 120 python tools/gpu_sanity_bn.py > gpurun_out/r2_sanity_bn.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fused-bn 0 > gpurun_out/r2_bench_nofuse.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fused-bn 1 > gpurun_out/r2_bench_fuse.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 --fused-bn 1 > $GRAFT_REPO_ROOT/gpurun_out/r2_prof.log 2>&1
