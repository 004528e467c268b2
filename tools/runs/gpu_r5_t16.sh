#!/bin/bash
# r5 t16: fused attention at BERT-base shapes: timing + PMC (instruction mix, waits)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 120 python3 tools/bench_attention.py > $O/r5t16_attn.txt 2>&1; rc=$?; cat $O/r5t16_attn.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/r5at_p$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/bench_attention.py 3 > $O/r5at_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/r5at_p$i.log; exit 1; }
done
echo pmc done
