#!/bin/bash
# A/B of the pipeline's extraction depth (bench.py --depth / --lanes / --lane-matchers, HW queues),
# interleaved, pipeline only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06dab}
mkdir -p "$OUT"; cd "$R" || exit 1
for rep in 1 2; do
  for cfg in "1|--depth 1 --lanes 2" "1|--depth 2 --lanes 3 --lane-matchers 0" "8|--depth 2 --lanes 3" "6|--depth 2 --lanes 3 --lane-matchers 0"; do
    q=${cfg%%|*}; a=${cfg#*|}
    echo "queues $q: $a" >> "$OUT/ab.txt"
    if [ "$q" = "1" ]; then
      timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline --steps 60 $a > "$OUT/run.json" 2>> "$OUT/err.txt" || exit 1
    else
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline --steps 60 $a > "$OUT/run.json" 2>> "$OUT/err.txt" || exit 1
    fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['phase_ms_per_step'].get('step_wall'))" "$OUT/run.json" >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
