#!/bin/bash
# r6 t1: driver-exact bench on HEAD (determinism vs BENCH_r05), kernel-trace profile, step PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/r6t1_bench.log 2>&1 || { tail -5 $O/r6t1_bench.log; exit 1; }
tail -1 $O/r6t1_bench.log
bash tools/gpu_prof.sh r6t1 resnet50 > $O/r6t1_prof.log 2>&1 || { tail -5 $O/r6t1_prof.log; exit 1; }
head -14 $O/r6t1_resnet50_summary.md
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
i=0
for P in "$P1" "$P2" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/r6pmc_p$i -o pmc -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --graph 0 --steps 2 --warmup 1 --comm-probe 0 --preflight 0 \
    > $O/r6pmc_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/r6pmc_p$i.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/diag/step_pmc_table.py $O/r6pmc_p1 $O/r6pmc_p2 $O/r6pmc_p3 $O/r6pmc_p4 --top 45 > $O/r6_conv_pmc_raw.md && head -30 $O/r6_conv_pmc_raw.md
