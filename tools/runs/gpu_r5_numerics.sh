#!/bin/bash
# r5: per-layer engine gradient vs stock f32, component bisect of the lr-0.1 drift (tools/diag/engine_numerics.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O; D=/tmp/kf_num
export KUNGFU_DEV_KNOBS=1
timeout -k 10 300 python -u tools/diag/engine_numerics.py ref $D > $O/num_ref.log 2>&1 || { tail -30 $O/num_ref.log; exit 1; }
grep -E "^S|TRAJ" $O/num_ref.log
v() {  # tag, args / env...
  tag=$1; shift; args=""
  while [ "${1:0:2}" = "--" ]; do args="$args $1"; shift; done
  env "$@" timeout -k 10 240 python -u tools/diag/engine_numerics.py var $D $tag $args > $O/num_$tag.log 2>&1 || { tail -30 $O/num_$tag.log; return 1; }
  grep -E "^==|TRAJ|> 2x" $O/num_$tag.log
}
v engine && v noshadow --no-shadow && v nofused KUNGFU_FUSED_BLOCK=0 && v nowgrad KUNGFU_WGRAD=0 KUNGFU_WGRAD_RECT=0 \
  && v nostem KUNGFU_STEM=0 && v tiles1 KUNGFU_CONV_TILE_RULES=1 && v stockmod --stock-modules \
  && v nofused_noconv KUNGFU_FUSED_BLOCK=0 KUNGFU_CONV3X3=0 KUNGFU_CONV_RECT=0 \
  && v optonly --stock-modules --no-shadow KUNGFU_FUSED_BLOCK=0 KUNGFU_CONV3X3=0 KUNGFU_CONV_RECT=0 KUNGFU_WGRAD=0 KUNGFU_WGRAD_RECT=0 KUNGFU_STEM=0
