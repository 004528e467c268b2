#!/bin/bash
# VGG-16: fused-stack eligibility fix -- tests, eager bench, graph bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
j() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"), d["config"].get("final_loss"), d.get("verify",{}).get("replicas_consistent"))'; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "vgg or VGG" > $O/r4t27_tests.log 2>&1 || { tail -30 $O/r4t27_tests.log; exit 1; }
tail -2 $O/r4t27_tests.log
timeout -k 10 300 python bench.py --model vgg16 --steps 20 --warmup 5 > $O/r4t27_vgg16.log 2>&1 || { tail -5 $O/r4t27_vgg16.log; exit 1; }
echo "vgg16 default $(tail -1 $O/r4t27_vgg16.log | j)"
timeout -k 10 300 python bench.py --model vgg16 --graph 1 --steps 20 --warmup 5 > $O/r4t27_vgg16_g.log 2>&1 || { tail -5 $O/r4t27_vgg16_g.log; exit 1; }
echo "vgg16 graph $(tail -1 $O/r4t27_vgg16_g.log | j)"
