#!/bin/bash
# round-end rehearsal: the whole GPU suite, smoke(), the default bench (as the driver runs them), plus the
# other models' default benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O; TAG=${1:-r4final}
timeout -k 10 1000 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > $O/${TAG}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/${TAG}_pytest.log | head -20; tail -1 $O/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { tail -20 $O/${TAG}_smoke.log; exit 1; }
tail -1 $O/${TAG}_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${TAG}_bench.log 2>&1 || exit $?
tail -1 $O/${TAG}_bench.log | cut -c1-300
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
for M in inception_v3 vgg16 bert_base; do
  OPT=ssgd; [ $M = bert_base ] && OPT=gns
  timeout -k 10 300 python bench.py --model $M --optimizer $OPT --steps 20 --warmup 5 > $O/${TAG}_$M.log 2>&1 || exit 1
  echo "$M $(tail -1 $O/${TAG}_$M.log | j)"
done
