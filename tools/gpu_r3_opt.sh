#!/bin/bash
# Configs 3/4 on one GPU: forced-comm SMA (1-rank RCCL model all-reduce on
# the comm stream) and prefetched pair averaging (self-pull through the IPC store on a copy
# stream) vs S-SGD: throughput + kernel/copy traces with overlap tables.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/kungfu_amd/tuning/miopen
for o in ssgd sma pair; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --optimizer $o > "$OUT/r3o_bench_$o.log" 2>&1 || exit $?
  echo "$o $(tail -1 $OUT/r3o_bench_$o.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["comm"])')"
done
cd /tmp && export TMPDIR=/tmp
for o in sma pair; do
  timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/r3o_${o}_prof" -o prof --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --optimizer $o --steps 6 --warmup 3 > "$OUT/r3o_${o}_prof.log" 2>&1 || exit $?
  T="$OUT/r3o_${o}_prof/prof_kernel_trace.csv"; C="$OUT/r3o_${o}_prof/prof_memory_copy_trace.csv"
  CP=""; [ -f "$C" ] && CP="--copies $C"
  RE='ncclDevKernel|rccl|oneRank|nccl|memcpy|copyBuffer|Copy'
  python3 "$GRAFT_REPO_ROOT/tools/prof_overlap.py" "$T" --comm-regex "$RE" $CP > "$OUT/r3o_${o}_overlap.md" 2>&1
  python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$T" --top 30 --marker sgd > "$OUT/r3o_${o}_summary.md" 2>&1
  cat "$OUT/r3o_${o}_overlap.md"
done
