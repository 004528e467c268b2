#!/bin/bash
# r5 t15: per-kernel HBM roofline of a ResNet-50 step (two PMC passes, eager) + the graph bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/r5rl_p$i -o pmc -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --graph 0 --steps 2 --warmup 1 --comm-probe 0 --preflight 0 \
    > $O/r5rl_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/r5rl_p$i.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/diag/roofline_table.py $O/r5rl_p1 $O/r5rl_p2 > $O/r5_resnet50_roofline.md && head -60 $O/r5_resnet50_roofline.md
