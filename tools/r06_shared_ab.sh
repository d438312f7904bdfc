#!/bin/bash
# Pipeline A/B: the default (depth 1, 2 lanes) vs batch k+1's extraction queued behind batch k's on
# one shared extractor stream (--depth 2 --shared-ex-stream 1), interleaved, pipeline only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06sh}
mkdir -p "$OUT"; cd "$R" || exit 1
for rep in 1 2; do
  for a in "--depth 1" "--depth 2 --shared-ex-stream 1" "--depth 1 --shared-ex-stream 1"; do
    echo "$a" >> "$OUT/ab.txt"
    timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline --steps 60 $a > "$OUT/run.json" 2>> "$OUT/err.txt" || { tail -20 "$OUT/err.txt"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['phase_ms_per_step'].get('step_wall'), d.get('stage_ms_per_step'))" "$OUT/run.json" >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
