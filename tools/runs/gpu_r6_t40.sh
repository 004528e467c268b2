#!/bin/bash
# r6 t40: BERT-base linear weight gradients: every split-K tile variant x split count vs the plan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u tools/bench_linear_wgrad.py --sweep > $O/r6t40_lin.log 2>&1 || { tail -5 $O/r6t40_lin.log; exit 1; }
cat $O/r6t40_lin.log | grep -v "^/opt"
