set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn or bottleneck or finalize or resnet or inception" > $O/fin_t.log 2>&1; echo "tests rc=$? $(tail -1 $O/fin_t.log)"
for i in 1 2; do timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/fin_b$i.log 2>&1 || exit 1; python -c "import json,sys;d=json.loads(open('$O/fin_b$i.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"; done
bash tools/gpu_prof.sh r3fin resnet50 | grep -E "finalize|kernel sum|wall"
