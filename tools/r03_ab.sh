#!/bin/bash
# Round-3 A/B pass: the pose / BA parity tests on the in-tree library, k_pose_opt A/B between two
# library builds, the global-BA solve with the one-wave-per-node sweeps (ORBGPU_LDLT_SWEEP=1)
# against the node-parallel ones, and the pose kernel's wave-state counters.
# usage: bash tools/r03_ab.sh <tag> <libA.so> <libB.so>
set -o pipefail
TAG=${1:-ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_pose.py tests/test_gpu_frame_ops.py tests/test_gpu_ba_g2o_order.py \
  tests/test_gpu_track_local_map.py tests/test_gpu_ba_units.py tests/test_gpu_ba_sharded.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
bash tools/pose_ab.sh "$TAG/pose" "$2" "$3" || exit 1
for v in 1 0; do
  ORBGPU_LDLT_SWEEP=$v timeout -k 10 200 python3 tools/gba_timing.py 2000:0 2000:4 > "$OUT/gba_sweep$v.txt" 2>&1 || { tail -5 "$OUT/gba_sweep$v.txt"; exit 1; }
  echo "sweep=$v"; cat "$OUT/gba_sweep$v.txt"
done
bash tools/pose_stall.sh "$TAG/stall" || exit 1
