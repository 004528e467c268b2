#!/bin/bash
# the driver's round-end GPU checks: the whole GPU suite (-x) and smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O; TAG=${1:-r5suite}
timeout -k 10 1080 python -u -m pytest tests -x -v --timeout 600 --timeout-method thread -m gpu > $O/${TAG}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/${TAG}_pytest.log | head -20; tail -1 $O/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { tail -20 $O/${TAG}_smoke.log; exit 1; }
tail -1 $O/${TAG}_smoke.log
