#!/bin/bash
# Local BA (config 4) single-stream A/B of environment knobs, interleaved (three rounds), then
# one phase breakdown per knob (ORBGPU_BA_TIMES=1).
# usage: bash tools/r06_lba_ab.sh <tag> "ENV=..|label" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06lab}
shift
mkdir -p "$OUT"; cd "$R" || exit 1
for rep in 1 2 3; do
  for cfg in "$@"; do
    envs=${cfg%%|*}; label=${cfg#*|}
    printf "%s: " "$label" >> "$OUT/ab.txt"
    env $envs timeout -k 10 120 python tools/ba_timing.py 40 2>> "$OUT/err.txt" | grep "^gpu:" >> "$OUT/ab.txt" || { tail -20 "$OUT/err.txt"; exit 1; }
  done
done
for cfg in "$@"; do
  envs=${cfg%%|*}; label=${cfg#*|}
  echo "== $label" >> "$OUT/phases.txt"
  env $envs ORBGPU_BA_TIMES=1 timeout -k 10 120 python tools/ba_timing.py 3 >> "$OUT/phases.txt" 2>&1 || exit 1
done
cat "$OUT/ab.txt"
