#!/bin/bash
# Kernel stats of ONE extractor (tools/extract_timing.py, B=64) under rocprofv3: bash tools/prof_extract.sh <tag>
set -o pipefail
TAG=${1:-pe}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o ex -- python3 "$R/tools/extract_timing.py" 64 \
  > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
grep -v amdgpu.ids "$OUT/prof.log" | tail -2
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 12
