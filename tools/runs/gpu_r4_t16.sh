#!/bin/bash
# hipBLASLt solution tuning for BERT-base's GEMMs (PyTorch TunableOp): tune once, then A/B the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
export PYTORCH_TUNABLEOP_VERBOSE=1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_bert.csv \
  timeout -k 10 600 python -u bench.py --model bert_base --optimizer gns --steps 3 --warmup 2 > $O/r4t16_tune.log 2>&1 || { tail -30 $O/r4t16_tune.log; exit 1; }
tail -3 $O/r4t16_tune.log | cut -c1-300; ls -la $O/tunableop_bert*.csv; wc -l $O/tunableop_bert*.csv
F=$(ls $O/tunableop_bert*.csv | head -1)
for T in 1 0 1 0; do
  if [ $T = 1 ]; then
    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$F timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t16_bert_t$T.log 2>&1 || { tail -20 $O/r4t16_bert_t$T.log; exit 1; }
  else
    timeout -k 10 300 python bench.py --model bert_base --optimizer gns --steps 30 --warmup 6 > $O/r4t16_bert_t$T.log 2>&1 || { tail -20 $O/r4t16_bert_t$T.log; exit 1; }
  fi
  echo "bert tunableop=$T $(tail -1 $O/r4t16_bert_t$T.log | j)"
done
