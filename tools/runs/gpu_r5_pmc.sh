#!/bin/bash
# PMC passes over BERT-base's GEMMs: hipBLASLt vs gemm_nt, forward and data gradient, 4 shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
P3="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM"
for S in 0 1 2 3; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/r5pmc_s${S}_p$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/diag/gemm_pmc.py $S > $O/r5pmc_s${S}_p$i.log 2>&1 || { echo "shape $S pass $i failed"; tail -5 $O/r5pmc_s${S}_p$i.log; exit 1; }
  done
done
python3 $GRAFT_REPO_ROOT/tools/diag/gemm_pmc_table.py $O > $O/r5_gemm_pmc.md && cat $O/r5_gemm_pmc.md
