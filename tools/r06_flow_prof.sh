#!/bin/bash
# k_pyr_flow vs per-level launches: extractor stage times (128 and 2 images) and a kernel trace of
# the 128-image case for each; then k_ldlt_panel's chunk barrier vs barrier per pivot (global BA
# timing + kernel stats).  usage: bash tools/r06_flow_prof.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06fp}
mkdir -p "$OUT"; cd "$R" || exit 1
export TMPDIR=/tmp
for F in 1 0; do
  for B in 128 2; do
    echo "B=$B flow=$F: $(ORBGPU_PYR_FLOW=$F timeout -k 10 120 python tools/extract_timing.py $B 2>/dev/null | tail -1)" | tee -a "$OUT/extract_ab.txt" || exit 1
  done
  ORBGPU_PYR_FLOW=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof$F" -o ex -- python3 tools/extract_timing.py 128 > /dev/null 2>&1 || exit 1
  python3 tools/prof_csv.py "$(find "$OUT/prof$F" -name '*kernel_stats.csv' | head -1)" 12 > "$OUT/kernel_stats_flow$F.txt"
  python3 tools/timeline.py "$(find "$OUT/prof$F" -name '*kernel_trace.csv' | head -1)" 8 > "$OUT/timeline_flow$F.txt"
  cat "$OUT/kernel_stats_flow$F.txt"; head -30 "$OUT/timeline_flow$F.txt"
  rm -rf "$OUT/prof$F"
done
for P in 0 1 0 1; do
  echo "panel sync $P: $(ORBGPU_LDLT_PANEL_SYNC=$P timeout -k 10 300 python tools/gba_timing.py 2000:4 2>&1 | grep nkf)" | tee -a "$OUT/panel_ab.txt" || exit 1
done
for P in 0 1; do
  ORBGPU_LDLT_PANEL_SYNC=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gprof$P" -o g -- python3 tools/gba_timing.py 2000:4 > /dev/null 2>&1 || exit 1
  python3 tools/prof_csv.py "$(find "$OUT/gprof$P" -name '*kernel_stats.csv' | head -1)" 8 > "$OUT/gba_stats_sync$P.txt"
  cat "$OUT/gba_stats_sync$P.txt"
  rm -rf "$OUT/gprof$P"
done
