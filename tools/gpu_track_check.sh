#!/bin/bash
# Tracking-lane pass on the GPU box: the parity tests of the lane's calls (matching, stereo, pose,
# frame ops, TrackLocalMap, g2o-order pose), then the pipeline timeline (tools/gpu_timeline.sh).
# usage: bash tools/gpu_track_check.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-tc}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pose.py tests/test_gpu_frame_ops.py tests/test_gpu_track_local_map.py \
  tests/test_gpu_match.py tests/test_gpu_stereo.py tests/test_gpu_ba_g2o_order.py -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash tools/gpu_timeline.sh "$TAG" "$@"
