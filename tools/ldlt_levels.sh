#!/bin/bash
# Level-by-level launches of one sparse LDL^T solve of BundleAdjustment at 2,000 keyframes (4 laps).
# usage: bash tools/ldlt_levels.sh <tag> [kf:laps]
set -o pipefail
TAG=${1:-ll}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/prof" -o gba -- python3 tools/gba_timing.py "${2:-2000:4}" \
  > "$OUT/gba_timing.txt" 2>&1 || { tail -20 "$OUT/gba_timing.txt"; exit 1; }
grep "nkf" "$OUT/gba_timing.txt"
python3 tools/ldlt_levels.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" > "$OUT/levels.txt"
rm -rf "$OUT/prof"
cat "$OUT/levels.txt"
