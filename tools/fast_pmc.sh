#!/bin/bash
# k_fast_cells roofline evidence: FETCH_SIZE, WRITE_SIZE and SQ_INSTS_VALU/SQ_WAVES passes over the
# bench's roofline workload (tools/extract_timing.py 64), per-launch json -> gpurun_out/<tag>/;
# copy traffic.json / valu.json to profiles/traffic_r03.json / valu_r03.json afterwards.
# usage: bash tools/fast_pmc.sh <tag>
set -o pipefail
TAG=${1:-fp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES"; do
  d=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -f csv -d "$OUT/$d" -o ex -- python3 "$R/tools/extract_timing.py" 64 \
    > "$OUT/$d.log" 2>&1 || { echo "$c pass failed"; tail -20 "$OUT/$d.log"; exit 1; }
done
W="workload: tools/extract_timing.py 64 = the bench roofline pass (left batch, seed 1000, B=64)"
python3 tools/pmc_traffic.py "$(find "$OUT/FETCH_SIZE" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT/WRITE_SIZE" -name '*counter_collection.csv' | head -1)" "$OUT/traffic.json" "$W" || exit 1
python3 tools/pmc_valu.py "$(find "$OUT/SQ_INSTS_VALU" -name '*counter_collection.csv' | head -1)" "$OUT/valu.json" "$W" || exit 1
rm -rf "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE" "$OUT/SQ_INSTS_VALU"
python3 -c "import json; t=json.load(open('$OUT/traffic.json')); v=json.load(open('$OUT/valu.json')); print({k: t[k] for k in t if 'fast' in k}); print({k: v[k] for k in v if 'fast' in k})"
