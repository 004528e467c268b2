#!/bin/bash
# r6 t14: which kernels the hardware bf16 conversion slowed down: BERT kernel traces, hw vs soft .so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
SO=kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_hip_hw.so
export TMPDIR=/tmp
for V in hw soft; do
  if [ $V = hw ]; then cp /tmp/_hip_hw.so $SO; else cp build_ab/_hip_soft.so $SO; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6t14_$V -o kt --output-format csv -- python3 bench.py --model bert_base --optimizer gns --steps 4 --warmup 2 > $O/r6t14_$V.log 2>&1 || { tail -5 $O/r6t14_$V.log; exit 1; }
  echo "$V done"
done
cp /tmp/_hip_hw.so $SO
