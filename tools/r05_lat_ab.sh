#!/bin/bash
# Batch-1 latency A/B (bench.py --latency-only), variants "<label>|<env>|<args>" interleaved, three
# rounds; prints device and host-path p50 / mean per run.
# usage: bash tools/r05_lat_ab.sh <tag> "<label>|<env>|<args>" ...
set -o pipefail
TAG=$1; shift
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
for round in 1 2 3; do
  for V in "$@"; do
    IFS='|' read -r LABEL ENVS ARGS <<< "$V"
    env $ENVS timeout -k 10 300 python bench.py --latency-only $ARGS > "$OUT/lat_${LABEL}_$round.json" 2> "$OUT/lat_${LABEL}_$round.err" \
      || { tail -20 "$OUT/lat_${LABEL}_$round.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['latency']; h=d['host_path']; print(sys.argv[2], sys.argv[3], 'device p50', d['p50_ms'], 'mean', d['mean_ms'], '| host p50', h['p50_ms'], 'mean', h['mean_ms'], 'max', max(h['frame_ms'][2:]))" "$OUT/lat_${LABEL}_$round.json" "$round" "$LABEL" | tee -a "$OUT/ab.txt"
  done
done
