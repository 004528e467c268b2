#!/bin/bash
# r6 t20: what limits the stride-1 3x3 convs?  counter list + SQ / TA / TD / TCP passes on the isolated shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 120 python tools/bench_conv3x3_s1.py -1 0 1 2 7 > $O/r6t20_times.log 2>&1 || { tail -5 $O/r6t20_times.log; exit 1; }
cat $O/r6t20_times.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/r6t20_counters.txt 2>&1 || { echo "list failed"; tail -3 $O/r6t20_counters.txt; }
have() { grep -q "\b$1\b" $O/r6t20_counters.txt && echo $1; }
PA="$(have TA_TA_BUSY_sum) $(have TA_BUFFER_READ_WAVEFRONTS_sum) GRBM_GUI_ACTIVE GRBM_COUNT"
PB="$(have TD_TD_BUSY_sum) $(have TCP_PENDING_STALL_CYCLES_sum) $(have TCP_TCR_TCP_STALL_CYCLES_sum) $(have TCP_READ_TAGCONFLICT_STALL_CYCLES_sum) $(have TCP_TCC_READ_REQ_LATENCY_sum)"
PC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
echo "PA=$PA"; echo "PB=$PB"
i=0
for P in "$PC" "$PA" "$PB"; do
  i=$((i+1))
  ITERS=3 timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/r6t20_p$i -o pmc -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_conv3x3_s1.py > $O/r6t20_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/r6t20_p$i.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, os, sys, collections
o = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for i in (1, 2, 3):
    for f in glob.glob(os.path.join(o, "r6t20_p%d" % i, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv_kernel" not in r["Kernel_Name"]:
                continue
            key = (r["Kernel_Name"].split("(")[0][-40:], r["Grid_Size"] if "Grid_Size" in r else r.get("Grid_Size_X", ""))
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
