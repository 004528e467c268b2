#!/bin/bash
# round-end rehearsal, part B: every other GPU test file, smoke(), the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O; TAG=${1:-r4fb}
timeout -k 10 900 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu --ignore tests/test_gpu.py > $O/${TAG}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/${TAG}_pytest.log | head -20; tail -2 $O/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { tail -20 $O/${TAG}_smoke.log; exit 1; }
tail -1 $O/${TAG}_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${TAG}_bench.log 2>&1 || exit $?
tail -1 $O/${TAG}_bench.log | cut -c1-400
