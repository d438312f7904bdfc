#!/bin/bash
# Extraction kernels under rocprofv3 (round 5): the extraction tests, then stage timings and kernel
# stats of one extractor at 128 and 2 images: per-level pyramid launches (chain off) and the
# chained pyramid tail from each level given.
# usage: bash tools/r05_extract_prof.sh <tag> [from-level ...]
set -o pipefail
TAG=${1:-r05p}
shift
FROMS=${*:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_extract.txt" 2>&1 \
  || { tail -30 "$OUT/pytest_extract.txt"; exit 1; }
tail -1 "$OUT/pytest_extract.txt"
for F in 0 $FROMS; do
  C=1; [ "$F" = 0 ] && C=0
  for B in 128 2; do
    echo "B=$B chain=$C from=$F: $(ORBGPU_PYR_CHAIN=$C ORBGPU_PYR_CHAIN_FROM=$F timeout -k 10 120 python tools/extract_timing.py $B 2>/dev/null | tail -1)" | tee -a "$OUT/extract_ab.txt" || exit 1
  done
  ORBGPU_PYR_CHAIN=$C ORBGPU_PYR_CHAIN_FROM=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof$F" -o ex -- python3 tools/extract_timing.py 128 > /dev/null 2>&1 || exit 1
  KS=$(find "$OUT/prof$F" -name '*kernel_stats.csv' | head -1)
  KT=$(find "$OUT/prof$F" -name '*kernel_trace.csv' | head -1)
  python3 tools/prof_csv.py "$KS" 12 > "$OUT/kernel_stats_from$F.txt"
  python3 tools/timeline.py "$KT" 8 > "$OUT/timeline_from$F.txt"
  cat "$OUT/kernel_stats_from$F.txt" "$OUT/timeline_from$F.txt"
  rm -rf "$OUT/prof$F"
done
