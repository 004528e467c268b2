#!/bin/bash
# r5 t12: row-image wgrad: per-shape timing (variants 6 / 8) + PMC passes on the narrow stem shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wgrad_rows.py > $O/r5t12_pytest.log 2>&1
rc=$?; tail -1 $O/r5t12_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_inception_wgrad.py > $O/r5t12_wgrad.txt 2>&1 || exit 1
grep -E "rows" $O/r5t12_wgrad.txt
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
P3="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM"
for S in 0 2; do for V in 6 10; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/r5wr_s${S}_v${V}_p$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/diag/wgrad_rows_pmc.py $S $V > $O/r5wr_s${S}_v${V}_p$i.log 2>&1 || { echo "shape $S v $V pass $i failed"; tail -5 $O/r5wr_s${S}_v${V}_p$i.log; exit 1; }
  done
done; done
echo pmc done
