#!/bin/bash
# Round-end rehearsal on one MI355X: full GPU suite, smoke(), the default bench (as the driver runs it).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-final}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -2 "$OUT/${TAG}_pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || { tail -20 "$OUT/${TAG}_smoke.log"; exit 1; }
tail -1 "$OUT/${TAG}_smoke.log"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bench.log"
