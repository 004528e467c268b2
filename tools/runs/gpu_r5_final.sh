#!/bin/bash
# round-5 rehearsal of the driver's round-end checks: GPU suite (-x), smoke(), then every model's bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O; TAG=${1:-r5final}
timeout -k 10 1080 python -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu > $O/${TAG}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/${TAG}_pytest.log | head -20; tail -1 $O/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { tail -20 $O/${TAG}_smoke.log; exit 1; }
tail -1 $O/${TAG}_smoke.log
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python bench.py > $O/${TAG}_resnet50.log 2>&1 || { tail -5 $O/${TAG}_resnet50.log; exit 1; }
echo "resnet50 (default): $(tail -1 $O/${TAG}_resnet50.log | j)"
for M in inception_v3 vgg16; do
  timeout -k 10 300 python bench.py --model $M --steps 20 --warmup 6 > $O/${TAG}_$M.log 2>&1 || { tail -5 $O/${TAG}_$M.log; exit 1; }
  echo "$M: $(tail -1 $O/${TAG}_$M.log | j)"
done
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/${TAG}_bert.log 2>&1 || { tail -5 $O/${TAG}_bert.log; exit 1; }
echo "bert_base gns: $(tail -1 $O/${TAG}_bert.log | j)"
