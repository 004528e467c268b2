#!/bin/bash
# r6 t23: PMC passes over the 56x56 64->64 3x3 conv: tap-wise (v2) vs row-image (v24)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
PB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
PC="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum FETCH_SIZE"
for v in 2 24; do
  i=0
  for P in "$PA" "$PB" "$PC"; do
    i=$((i+1))
    SHAPES=0 ITERS=3 timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/r6t23_v${v}_p$i -o pmc -- \
      python3 $GRAFT_REPO_ROOT/tools/bench_conv3x3_s1.py $v > $O/r6t23_v${v}_p$i.log 2>&1 || { echo "pass $v $i failed"; tail -5 $O/r6t23_v${v}_p$i.log; exit 1; }
  done
done
echo ok
