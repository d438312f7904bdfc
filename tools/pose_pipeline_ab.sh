#!/bin/bash
# Pipeline A/B of two library builds: pose kernel alone (tools/pose_timing.py 63) and the bench
# pipeline line (no CPU baselines), alternating A B A B.  usage: bash tools/pose_pipeline_ab.sh <tag> <libA> <libB>
set -o pipefail
TAG=${1:-pab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
for rep in 1 2; do
  for lib in "$2" "$3"; do
    n=$(basename "$lib" .so)
    ORBGPU_LIB="$lib" timeout -k 10 120 python3 tools/pose_timing.py 63 > "$OUT/$n.pose$rep.txt" 2>&1 || { tail -5 "$OUT/$n.pose$rep.txt"; exit 1; }
    ORBGPU_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu-baseline --pipeline-only --steps 40 > "$OUT/$n.$rep.json" 2> "$OUT/$n.$rep.err" || { tail -5 "$OUT/$n.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], open(sys.argv[3]).read().strip())" "$OUT/$n.$rep.json" "$n" "$OUT/$n.pose$rep.txt"
  done
done
