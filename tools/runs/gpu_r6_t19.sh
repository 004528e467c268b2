#!/bin/bash
# r6 t19: ResNet-50 A/B of the in-launch BN finalize (fused_block._INLAUNCH_FIN), two interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 8 --comm-probe 0 > $O/r6t19_base_$r.log 2>&1 || { tail -5 $O/r6t19_base_$r.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('base',d['ms_per_step'],d['config']['final_loss'])" $O/r6t19_base_$r.log
  timeout -k 10 300 python tools/bench_switch.py kungfu_amd.ops.fused_block:_INLAUNCH_FIN=True -- --steps 30 --warmup 8 --comm-probe 0 > $O/r6t19_fin_$r.log 2>&1 || { tail -5 $O/r6t19_fin_$r.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('inlaunch_fin',d['ms_per_step'],d['config']['final_loss'])" $O/r6t19_fin_$r.log
done
