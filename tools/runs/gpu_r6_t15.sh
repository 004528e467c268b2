#!/bin/bash
# r6 t15: integer bf16 rounding everywhere (in-tree .so) vs the same with v_cvt_pk_bf16_f32 still in
# attention / stem / stem3 (build_ab/_hip_soft.so, r6t13's "soft"): BERT + ResNet-50, then stem/attention tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
SO=kungfu_amd/_hip.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_hip_all.so
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])'; }
for i in 1 2; do
  for V in all part; do
    if [ $V = all ]; then cp /tmp/_hip_all.so $SO; else cp build_ab/_hip_soft.so $SO; fi
    timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > $O/r6t15_bert_${V}_$i.log 2>&1 || { tail -5 $O/r6t15_bert_${V}_$i.log; exit 1; }
    echo "bert $V run $i: $(tail -1 $O/r6t15_bert_${V}_$i.log | j)"
    timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/r6t15_r50_${V}_$i.log 2>&1 || { tail -5 $O/r6t15_r50_${V}_$i.log; exit 1; }
    echo "r50 $V run $i: $(tail -1 $O/r6t15_r50_${V}_$i.log | j)"
  done
done
cp /tmp/_hip_all.so $SO
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "stem or attention" > $O/r6t15_pytest.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/r6t15_pytest.log | tail -4; exit $rc
