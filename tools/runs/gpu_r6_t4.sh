#!/bin/bash
# r6 t4: interleaved tile sweep; bench A/B: wgrad on the side stream (graph branches) vs inline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for i in 1 2; do
  for V in 0 1; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 8 --wgrad-side $V > $O/r6t4_side${V}_$i.log 2>&1 || { tail -5 $O/r6t4_side${V}_$i.log; exit 1; }
    echo "wgrad-side $V run $i: $(tail -1 $O/r6t4_side${V}_$i.log | j)"
  done
done
timeout -k 10 900 python tools/bench_conv_tiles.py > $O/r6t4_tiles.log 2>&1; rc=$?
grep -v amdgpu.ids $O/r6t4_tiles.log
exit $rc
