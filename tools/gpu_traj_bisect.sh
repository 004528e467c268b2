#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export KUNGFU_DEV_KNOBS=1  # A/B of developer knobs (kungfu_amd/knobs.py)
OUT=gpurun_out; mkdir -p $OUT
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -s --timeout 280 --timeout-method thread -k resnet50_full_size > $OUT/traj_$tag.log 2>&1
  echo "$tag rc=$? $(grep -E 'lr0.1 engine' $OUT/traj_$tag.log | cut -c1-200)"
}
run off KUNGFU_CONV_STAGGER=0 KUNGFU_CONV_TILE_RULES=1 KUNGFU_WROWS_STAGGER=0
run def
run stag_only KUNGFU_CONV_TILE_RULES=1 KUNGFU_WROWS_STAGGER=0
