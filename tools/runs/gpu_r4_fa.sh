#!/bin/bash
# round-end rehearsal, part A: tests/test_gpu.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O; TAG=${1:-r4fa}
timeout -k 10 1100 python -u -m pytest tests/test_gpu.py -v --timeout 300 --timeout-method thread -m gpu > $O/${TAG}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/${TAG}_pytest.log | head -20; tail -2 $O/${TAG}_pytest.log; exit $rc
