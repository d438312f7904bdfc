#!/bin/bash
# Host-IO leg A/B: the step's H2D copy on 1 / 2 / 4 copy streams (pipeline-only line, interleaved).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06h2d}
mkdir -p "$OUT"; cd "$R" || exit 1
for rep in 1 2; do
  for k in 1 2 4; do
    timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline --steps 60 --h2d-streams $k > "$OUT/run.json" 2>> "$OUT/err.txt" || { tail -20 "$OUT/err.txt"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); h=d['value_host_io']; print('h2d streams', sys.argv[2], d['value'], h['value'], h['h2d_GBps_achieved'], round(h['value']/d['value'],3))" "$OUT/run.json" $k >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
