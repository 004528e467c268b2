#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python tools/diag/grad_compare.py > $O/r4t3_gradcmp.log 2>&1; grep -v "rel 1\.\|rel 0\." $O/r4t3_gradcmp.log | tail -60
