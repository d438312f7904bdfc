#!/bin/bash
# Global BA (config 5: 2000 keyframes, 4 laps) on one GPU: timing, per-kernel stats of one
# BundleAdjustment(10) call and the per-level launches of its last sparse LDL^T solve.
# usage: bash tools/r05_gba_prof.sh <tag>
set -o pipefail
TAG=${1:-r05gbap}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
ORBGPU_BA_TIMES=1 timeout -k 10 300 python tools/gba_timing.py 2000:4 > "$OUT/gba_timing.txt" 2>&1 || { tail -20 "$OUT/gba_timing.txt"; exit 1; }
grep nkf "$OUT/gba_timing.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d "$OUT/prof" -o p -- python3 tools/gba_timing.py 2000:4 > "$OUT/prof.txt" 2>&1 || { tail -20 "$OUT/prof.txt"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 30 > "$OUT/gba_kernel_stats.txt"
python3 tools/ldlt_levels.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" > "$OUT/gba_ldlt_levels.txt"
python3 tools/gba_struct_timeline.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" "$(find "$OUT/prof" -name '*memory_copy_trace.csv' | head -1)" > "$OUT/gba_struct_timeline.txt"
head -32 "$OUT/gba_kernel_stats.txt"; tail -1 "$OUT/gba_ldlt_levels.txt"; tail -1 "$OUT/gba_struct_timeline.txt"
rm -rf "$OUT/prof"
