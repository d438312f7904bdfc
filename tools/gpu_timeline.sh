#!/bin/bash
# Pipeline timeline on the GPU box: rocprofv3 kernel + memory-copy trace of a short bench run
# (no CPU baselines, no BA/RANSAC legs' CPU work), the step-8 timeline and the kernel stats.
# usage: bash tools/gpu_timeline.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-tl}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
ORBGPU_LBA_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d "$OUT/prof" -o bench -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 20 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 40 > "$OUT/kernel_stats.txt"
python3 tools/timeline.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" 8 > "$OUT/timeline.txt"
cat "$OUT/timeline.txt"
head -45 "$OUT/kernel_stats.txt"
f=$(find "$OUT/prof" -name '*memory_copy_trace.csv' | head -1)
[ -n "$f" ] && cp "$f" "$OUT/memcpy_trace.csv"
exit 0
