#!/bin/bash
# Pipeline A/B (round 5): bench.py --pipeline-only for each variant, two alternating rounds.
# usage: bash tools/r05_pipe_ab.sh <tag> "<label>|<env>|<args>" ...
set -o pipefail
TAG=$1; shift
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
export TMPDIR=/tmp
for round in 1 2; do
  for V in "$@"; do
    IFS='|' read -r LABEL ENVS ARGS <<< "$V"
    L=$(env $ENVS timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline $ARGS 2> "$OUT/err_$LABEL.txt") || { tail -20 "$OUT/err_$LABEL.txt"; exit 1; }
    echo "$round $LABEL $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'])" "$L")" | tee -a "$OUT/ab.txt"
  done
done
