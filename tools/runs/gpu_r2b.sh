#!/bin/bash
# Round 2, second GPU pass: the new GPU tests (device graph plane host-staged, exact/skewed
# pair averaging, NaN propagation, BERT GNS numerics, full-size ResNet-50 numerics), then
# BERT-base S-SGD + gradient-noise-scale bench and a kernel trace of it (K5 kernels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2b}
mkdir -p "$OUT"
export MIOPEN_USER_DB_PATH=$PWD/kungfu_amd/tuning/miopen
timeout -k 10 700 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "graph or pair or nan or full_size or bert" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -60 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -3 "$OUT/${TAG}_pytest.log"
grep -E "^lr0" "$OUT/${TAG}_pytest.log" | head -4
timeout -k 10 400 python bench.py --model bert_base --optimizer gns --steps 20 --warmup 5 > "$OUT/${TAG}_bert.log" 2>&1 || { tail -30 "$OUT/${TAG}_bert.log"; exit 1; }
tail -1 "$OUT/${TAG}_bert.log"
timeout -k 10 400 python bench.py --model bert_base --optimizer ssgd --steps 20 --warmup 5 > "$OUT/${TAG}_bert_ssgd.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_bert_ssgd.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_bprof" -o prof --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model bert_base --optimizer gns --steps 6 --warmup 3 > "$OUT/${TAG}_bprof.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$OUT/${TAG}_bprof/prof_kernel_trace.csv" --marker adam --top 40 \
  > "$OUT/${TAG}_bprof_summary.md" 2>&1
head -50 "$OUT/${TAG}_bprof_summary.md"
