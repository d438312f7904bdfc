#!/bin/bash
# TrackLocalMap candidate search in the pipeline: per variant, two alternating bench.py
# --pipeline-only rounds (frames/s) and one rocprofv3 --stats run (the k_candidates launches'
# average duration beside the extraction grids).
# usage: bash tools/r05_cand_ab.sh <tag> "<label>|<env>" ...
set -o pipefail
TAG=$1; shift
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
export TMPDIR=/tmp
for round in 1 2; do
  for V in "$@"; do
    IFS='|' read -r LABEL ENVS <<< "$V"
    L=$(env $ENVS timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline 2> "$OUT/err_$LABEL.txt") || { tail -20 "$OUT/err_$LABEL.txt"; exit 1; }
    echo "$round $LABEL $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'])" "$L")" | tee -a "$OUT/ab.txt"
  done
done
for V in "$@"; do
  IFS='|' read -r LABEL ENVS <<< "$V"
  env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/p_$LABEL" -o p -- python3 bench.py --pipeline-only --no-cpu-baseline > /dev/null 2> "$OUT/perr_$LABEL.txt" || { tail -20 "$OUT/perr_$LABEL.txt"; exit 1; }
  python3 tools/prof_csv.py "$(find "$OUT/p_$LABEL" -name '*kernel_stats.csv' | head -1)" 40 > "$OUT/stats_$LABEL.txt"
  echo "$LABEL:"; grep "k_candidates\|k_select\|k_pose_opt" "$OUT/stats_$LABEL.txt" | tee -a "$OUT/ab.txt"
  rm -rf "$OUT/p_$LABEL"
done
