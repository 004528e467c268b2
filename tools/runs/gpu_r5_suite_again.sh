#!/bin/bash
# r5: the GPU suite once more on a fresh box (flake hunt before the round-end run; no -x: every failure listed)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O; TAG=${1:-r5again}
timeout -k 10 1080 python -u -m pytest tests -q --timeout 600 --timeout-method thread -m gpu > $O/${TAG}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/${TAG}_pytest.log | head -20; tail -1 $O/${TAG}_pytest.log; exit $rc
