#!/bin/bash
# Resize tile height A/B (round 5): extraction tests on the default library, then stage timings
# at 128 and 2 images and the step-8 kernel timeline for PT_H = 16 / 32 (default) / 64 builds.
set -o pipefail
TAG=${1:-r05pt}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_extract.txt" 2>&1 \
  || { tail -30 "$OUT/pytest_extract.txt"; exit 1; }
tail -1 "$OUT/pytest_extract.txt"
for V in 16 32 64; do
  LIBV=$R/build/liborbslam_gpu_pt$V.so; [ "$V" = 32 ] && LIBV=$R/c_orb_slam_amd/liborbslam_gpu.so
  for B in 128 2; do
    echo "PT_H=$V B=$B: $(ORBGPU_LIB=$LIBV timeout -k 10 120 python tools/extract_timing.py $B 2>/dev/null | tail -1)" | tee -a "$OUT/pt_ab.txt" || exit 1
  done
  ORBGPU_LIB=$LIBV timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/prof$V" -o ex -- python3 tools/extract_timing.py 128 > /dev/null 2>&1 || exit 1
  KT=$(find "$OUT/prof$V" -name '*kernel_trace.csv' | head -1)
  python3 tools/timeline.py "$KT" 8 > "$OUT/timeline_pt$V.txt"
  head -12 "$OUT/timeline_pt$V.txt"
  rm -rf "$OUT/prof$V"
done
