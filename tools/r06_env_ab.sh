#!/bin/bash
# Pipeline-only A/B of environment knobs, interleaved (two rounds).
# usage: bash tools/r06_env_ab.sh <tag> "ENV=..;bench args|label" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06env}
shift
mkdir -p "$OUT"; cd "$R" || exit 1
for rep in 1 2; do
  for cfg in "$@"; do
    spec=${cfg%%|*}; label=${cfg#*|}
    envs=${spec%%;*}; args=""
    [ "$spec" != "$envs" ] && args=${spec#*;}
    echo "$label ($envs / $args)" >> "$OUT/ab.txt"
    env $envs timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline --steps 60 $args > "$OUT/run.json" 2>> "$OUT/err.txt" || { tail -20 "$OUT/err.txt"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" "$OUT/run.json" >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
