#!/bin/bash
# r6 t29: the elastic BERT-GNS bench on the host data plane, 1 -> 2 ranks: default (bf16 wire) vs f32 wire
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
unset WORLD_SIZE RANK LOCAL_RANK MASTER_ADDR MASTER_PORT KUNGFU_SELF_SPEC
export KUNGFU_FORCE_DEVICE=0 KUNGFU_GPU_DATAPLANE=host PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 100 python -u bench.py --model bert_base --optimizer gns --elastic 1:3,2:4 --batch 8 --comm-dtype f32 > $O/r6t29_f32.log 2>&1; echo "f32 rc=$?"
tail -3 $O/r6t29_f32.log | cut -c1-300
timeout -k 10 100 python -u bench.py --model bert_base --optimizer gns --elastic 1:3,2:4 --batch 8 > $O/r6t29_auto.log 2>&1; echo "auto rc=$?"
tail -30 $O/r6t29_auto.log | cut -c1-300
