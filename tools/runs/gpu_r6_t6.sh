#!/bin/bash
# r6 t6: pipe vs conv_kernel bitwise; engine envelope test on main and on the no-pipe build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
SO=$(ls kungfu_amd/_hip*.so)
cp "$SO" /tmp/_hip_main.so
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q --timeout 120 --timeout-method thread -k "conv_pipe" > $O/r6t6_pipe.log 2>&1
echo "pipe tests: $(tail -1 $O/r6t6_pipe.log)"; grep -E "^FAILED|^E " $O/r6t6_pipe.log | head -10
for V in main nopipe; do
  [ $V = main ] && cp /tmp/_hip_main.so "$SO" || cp alt/_hip_$V.so "$SO"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -q -s --timeout 240 --timeout-method thread -k "envelope" > $O/r6t6_env_$V.log 2>&1
  echo "$V envelope: $(tail -1 $O/r6t6_env_$V.log)"; grep -E "loss f32" $O/r6t6_env_$V.log
done
cp /tmp/_hip_main.so "$SO"
