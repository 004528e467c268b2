#!/bin/bash
# Quick GPU check: selected GPU tests (-k expr), then optional bench.  Usage: bash tools/gpu_quick.sh TAG 'kexpr' [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; KEXPR=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 240 --timeout-method thread -k "$KEXPR" > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|^E " "$OUT/${TAG}_pytest.log" | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "$1" != "" ]; then
  timeout -k 10 300 python bench.py "$@" > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
  tail -1 "$OUT/${TAG}_bench.log" | cut -c1-300
fi
