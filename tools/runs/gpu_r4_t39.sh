#!/bin/bash
# ResNet-50 + emulated 8-rank all-reduces: kernel trace eager vs captured -> overlap of the comm kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for G in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/r4t39_g${G}_prof" -o prof --output-format csv -- \
    python3 "$R/bench.py" --graph $G --emulate-comm 8 --emulate-ctas 32 --steps 8 --warmup 4 > "$OUT/r4t39_g${G}.log" 2>&1 || exit $?
  echo "graph=$G $(python3 $R/tools/diag/emu_overlap.py $OUT/r4t39_g${G}_prof/prof_kernel_trace.csv --last-frac 0.4)"
done
