#!/bin/bash
# Round-5 A/B 5: extraction tests, then stage timings at 128 / 2 images per octree workgroup size
# and the octree's per-job durations (instrumented build).
set -o pipefail
TAG=${1:-r05ab5}
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_gpu_frame_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.txt" 2>&1 \
  || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for B in 128 2; do
  for T in 256 512; do
    echo "B=$B OCT_T=$T: $(ORBGPU_OCT_T=$T timeout -k 10 120 python tools/extract_timing.py $B 2>/dev/null | tail -1)" | tee -a "$OUT/oct_ab.txt" || exit 1
  done
  ORBGPU_LIB=$R0/build/liborbslam_gpu_prof5.so ORBGPU_PROF_DUMP=1 timeout -k 10 120 python tools/extract_timing.py $B > "$OUT/octree_jobs_B$B.txt" 2>&1 || { tail -20 "$OUT/octree_jobs_B$B.txt"; exit 1; }
  tail -3 "$OUT/octree_jobs_B$B.txt"
done
