#!/bin/bash
# PMC passes over gemm_nt vs hipBLASLt on BERT shapes (one counter group per run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
P3="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/r4pmc_$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/diag/gemm_pmc.py > $O/r4pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/r4pmc_$i.log; }
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out"
for f in sorted(glob.glob(O + "/r4pmc_*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        k = "gemm_nt<%s>" % k.split("<")[1].split(">")[0] if "gemm_nt" in k else ("blas" if "Cijk" in k else k[:40])
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", f.split("gpurun_out/")[1])
    for k, d in agg.items():
        print("  %-22s " % k + "  ".join("%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(d.items())))
PY
