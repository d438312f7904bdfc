#!/bin/bash
# Local BA on the GPU box: kernel + copy trace of tools/ba_timing.py (one problem at a time), the
# kernel stats and the timeline of the last call.  usage: bash tools/lba_prof.sh <tag> [reps]
set -o pipefail
TAG=${1:-lba}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ba_timing.py "${2:-40}" > "$OUT/timing.txt" 2>&1 || { tail -20 "$OUT/timing.txt"; exit 1; }
cat "$OUT/timing.txt"
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d "$OUT/prof" -o lba -- \
  python3 tools/ba_timing.py 10 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 20 > "$OUT/kernel_stats.txt"
python3 tools/lba_timeline.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" \
  "$(find "$OUT/prof" -name '*memory_copy_trace.csv' | head -1)" > "$OUT/timeline.txt"
head -22 "$OUT/kernel_stats.txt"
tail -1 "$OUT/timeline.txt"
