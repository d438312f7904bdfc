#!/bin/bash
# Round-5 A/B 4: extraction tests with the chained pyramid tail forced on, its stage timings at
# 128 / 2 images against the per-level launches, and the octree's per-job durations.
set -o pipefail
TAG=${1:-r05ab4}
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
export TMPDIR=/tmp
ORBGPU_PYR_CHAIN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_chain.txt" 2>&1 \
  || { tail -30 "$OUT/pytest_chain.txt"; exit 1; }
tail -1 "$OUT/pytest_chain.txt"
for B in 128 2; do
  for C in 0 1; do
    echo "B=$B chain=$C: $(ORBGPU_PYR_CHAIN=$C timeout -k 10 120 python tools/extract_timing.py $B 2>/dev/null | tail -1)" | tee -a "$OUT/chain_ab.txt" || exit 1
  done
  ORBGPU_LIB=$R0/build/liborbslam_gpu_prof5.so ORBGPU_PROF_DUMP=1 timeout -k 10 120 python tools/extract_timing.py $B > "$OUT/octree_jobs_B$B.txt" 2>&1 || { tail -20 "$OUT/octree_jobs_B$B.txt"; exit 1; }
  tail -3 "$OUT/octree_jobs_B$B.txt"
done
