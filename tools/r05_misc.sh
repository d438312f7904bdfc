#!/bin/bash
# Round-5 measurements beside the main check: the config-5 multi-GPU cost model (1/2/4/8
# in-process ranks under rocprofv3) and the octree's section timers at 2 and 128 images
# (instrumented build build/liborbslam_gpu_prof5.so).
set -o pipefail
TAG=${1:-r05m}
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_gpu_ba_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 \
  || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for B in 2 128; do
  ORBGPU_LIB=$R0/build/liborbslam_gpu_prof5.so ORBGPU_PROF_DUMP=1 timeout -k 10 120 python tools/extract_timing.py $B > "$OUT/octree_prof_B$B.txt" 2>&1 || { tail -20 "$OUT/octree_prof_B$B.txt"; exit 1; }
  cat "$OUT/octree_prof_B$B.txt"
done
bash tools/r05_gba_model.sh "$TAG/gba" 2000:4
