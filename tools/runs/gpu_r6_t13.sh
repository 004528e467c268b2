#!/bin/bash
# r6 t13: hardware (v_cvt_pk_bf16_f32) vs integer-trick bf16 rounding, same tree otherwise (build_ab/*.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
SO=kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_hip_hw.so
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "stem or inplace_residual" > $O/r6t13_pytest.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/r6t13_pytest.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_stem.py > $O/r6t13_stem.log 2>&1 || { tail -5 $O/r6t13_stem.log; exit 1; }
tail -5 $O/r6t13_stem.log
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for i in 1 2; do
  for V in hw soft; do
    if [ $V = hw ]; then cp /tmp/_hip_hw.so $SO; else cp build_ab/_hip_soft.so $SO; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/r6t13_${V}_$i.log 2>&1 || { tail -5 $O/r6t13_${V}_$i.log; exit 1; }
    echo "r50 $V run $i: $(tail -1 $O/r6t13_${V}_$i.log | j)"
  done
done
for V in hw soft; do
  if [ $V = hw ]; then cp /tmp/_hip_hw.so $SO; else cp build_ab/_hip_soft.so $SO; fi
  timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r6t13_bert_${V}.log 2>&1 || { tail -5 $O/r6t13_bert_${V}.log; exit 1; }
  echo "bert $V: $(tail -1 $O/r6t13_bert_${V}.log | j)"
done
cp /tmp/_hip_hw.so $SO
