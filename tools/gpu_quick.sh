#!/bin/bash
# Quick GPU pass: bench line without the CPU baselines, then a rocprofv3 kernel trace of the same
# command (kernel stats + step-8 timeline).  usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['phase_ms_per_step'], d['latency']['p50_ms'])" "$OUT/bench.json"
ORBGPU_LBA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline \
  > "$OUT/prof_bench.log" 2>&1 || { tail -30 "$OUT/prof_bench.log"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 40 > "$OUT/kernel_stats.txt"
python3 tools/timeline.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" 8 > "$OUT/timeline.txt"
cat "$OUT/timeline.txt"
