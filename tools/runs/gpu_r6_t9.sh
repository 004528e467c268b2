#!/bin/bash
# r6 t9: why is the BNP stem weight gradient slow: kernel trace + one PMC pass over tools/bench_stem.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6t9_kt -o kt -- python3 tools/bench_stem.py > $O/r6t9_kt.log 2>&1 || { tail -5 $O/r6t9_kt.log; exit 1; }
tail -8 $O/r6t9_kt.log
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD -d $O/r6t9_pmc -o pmc -- python3 tools/bench_stem.py > $O/r6t9_pmc.log 2>&1 || { tail -5 $O/r6t9_pmc.log; exit 1; }
echo pmc done
