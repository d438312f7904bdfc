#!/bin/bash
# Pipeline A/B of two bench.py argument sets on one build (no CPU baselines), alternating
# A B A B.  usage: bash tools/bench_ab.sh <tag> "<args A>" "<args B>"
set -o pipefail
TAG=${1:-bab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then a="$2"; else a="$3"; fi
    # shellcheck disable=SC2086
    timeout -k 10 300 python bench.py --no-cpu-baseline --pipeline-only --steps 60 $a > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" \
      || { tail -5 "$OUT/$v.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      "$OUT/$v.$rep.json" "$v($a)"
  done
done
