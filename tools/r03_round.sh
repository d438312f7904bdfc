#!/bin/bash
# One GPU pass for the round's tree: the whole -m gpu suite on the in-tree library, a k_pose_opt
# A/B of two builds with the pose parity tests on the second, and the pipeline timeline.
# usage: bash tools/r03_round.sh <tag> <libA.so> <libB.so>
set -o pipefail
TAG=${1:-rr}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_all.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_all.log"
[ $rc -eq 0 ] || exit $rc
bash tools/pose_ab.sh "$TAG/pose" "$2" "$3" || exit 1
ORBGPU_LIB="$R/$3" timeout -k 10 300 python -u -m pytest tests/test_gpu_pose.py tests/test_gpu_frame_ops.py \
  tests/test_gpu_ba_g2o_order.py tests/test_gpu_track_local_map.py tests/test_gpu_threads.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > "$OUT/pytest_pose_B.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_pose_B.log"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_timeline.sh "$TAG/tl" > "$OUT/timeline.log" 2>&1 || { tail -20 "$OUT/timeline.log"; exit 1; }
head -70 "$OUT/tl/timeline.txt"
