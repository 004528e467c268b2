#!/bin/bash
# r5 t28: MLM head micro-bench incl. split-K batched data gradient
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/bench_mlm_head.py > $O/r5t28_mlm.log 2>&1; rc=$?
grep -v amdgpu.ids $O/r5t28_mlm.log; exit $rc
