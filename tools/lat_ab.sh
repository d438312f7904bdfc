#!/bin/bash
# A/B of the batch-1 tracking latency legs (bench.py --latency-only), variants interleaved, two runs
# each.  usage: bash tools/lat_ab.sh <tag> "<bench args A>" "<bench args B>" ...
set -o pipefail
TAG=${1:-lat}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --latency-only $v > "$OUT/lat_v${i}_$rep.json" 2> "$OUT/lat_v${i}_$rep.err" \
      || { tail -20 "$OUT/lat_v${i}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['latency']; print(repr(sys.argv[2]), 'device p50', d['p50_ms'], 'mean', d['mean_ms'], 'rot err', d['max_rotation_error'], '| host path p50', d['host_path']['p50_ms'])" "$OUT/lat_v${i}_$rep.json" "$v"
  done
done
