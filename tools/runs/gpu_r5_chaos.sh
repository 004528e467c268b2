#!/bin/bash
# r5: lr-0.1 trajectory sensitivity (tools/diag/engine_numerics.py chaos) + the engine twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O; D=/tmp/kf_num
timeout -k 10 300 python -u tools/diag/engine_numerics.py ref $D > $O/num2_ref.log 2>&1 || { tail -30 $O/num2_ref.log; exit 1; }
grep -E "TRAJ" $O/num2_ref.log
timeout -k 10 300 python -u tools/diag/engine_numerics.py chaos $D > $O/num2_chaos.log 2>&1 || { tail -30 $O/num2_chaos.log; exit 1; }
grep -E "TRAJ" $O/num2_chaos.log
timeout -k 10 240 python -u tools/diag/engine_numerics.py var $D engine2 > $O/num2_engine.log 2>&1 || { tail -30 $O/num2_engine.log; exit 1; }
grep -E "TRAJ|> 2x" $O/num2_engine.log
