#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/bench_prebn.py > $O/r5t9_prebn.log 2>&1; rc=$?; grep -v "^/opt\|RCCL\|HIP v\|ROCm v\|Hostname\|Librccl" $O/r5t9_prebn.log; exit $rc
