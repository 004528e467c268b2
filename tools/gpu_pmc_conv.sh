#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group) over the MFMA 3x3 conv on VGG
# shapes, plus the variant sweep.  Counters: SQ (8 slots), TCC (4), GRBM (2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-pmc}
mkdir -p "$OUT"
true

cd /tmp && export TMPDIR=/tmp
for SH in 0 2 3; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    -d "$OUT/${TAG}_sq_$SH" -o p --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_vgg_conv.py" --shape $SH --variant -1 --iters 5 > "$OUT/${TAG}_sq_$SH.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$OUT/${TAG}_tcc_$SH" -o p --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_vgg_conv.py" --shape $SH --variant -1 --iters 5 > "$OUT/${TAG}_tcc_$SH.log" 2>&1 || exit $?
done
python3 - "$OUT" "$TAG" << 'PY'
import csv, glob, os, sys, collections
out, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(os.path.join(out, tag + "_*_*", "p_counter_collection.csv"))):
    rows = [r for r in csv.DictReader(open(f)) if "conv_kernel" in r.get("Kernel_Name", "")]
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in rows:
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(os.path.basename(os.path.dirname(f)), {k: round(v / max(n[k], 1), 1) for k, v in agg.items()})
PY
