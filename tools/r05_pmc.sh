#!/bin/bash
# Round-5 PMC evidence: the matcher / pose passes (FETCH_SIZE, WRITE_SIZE, SQ_INSTS_VALU over
# bench.py --passes-only -> match_pmc_r05.json) and the k_fast_cells passes (tools/extract_timing.py
# 64 -> traffic_r05.json, valu_r05.json); one counter set per rocprofv3 run.
# usage: bash tools/r05_pmc.sh <tag>   (copy gpurun_out/<tag>/*_r05.json to profiles/ afterwards)
set -o pipefail
TAG=${1:-r05pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  echo "[pmc] match $c" && date
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -f csv -d "$OUT/m$c" -o m -- python3 "$R/bench.py" --passes-only \
    > "$OUT/m$c.log" 2>&1 || { echo "$c pass failed"; tail -20 "$OUT/m$c.log"; exit 1; }
done
python3 tools/pmc_match.py "$(find "$OUT/mFETCH_SIZE" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT/mWRITE_SIZE" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT/mSQ_INSTS_VALU" -name '*counter_collection.csv' | head -1)" "$OUT/match_pmc_r05.json" \
  "workload: bench.py --passes-only (B=64 KITTI stereo batch, one extractor over 2B images: 5 isolated ComputeStereoMatches + SearchByProjection(Cur,Last,7) + PoseOptimization + 16 dense 1200x1200 tiles)" > /dev/null || exit 1
rm -rf "$OUT/mFETCH_SIZE" "$OUT/mWRITE_SIZE" "$OUT/mSQ_INSTS_VALU"
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES"; do
  d=$(echo $c | cut -d' ' -f1)
  echo "[pmc] fast $d" && date
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -f csv -d "$OUT/f$d" -o ex -- python3 "$R/tools/extract_timing.py" 64 \
    > "$OUT/f$d.log" 2>&1 || { echo "$c pass failed"; tail -20 "$OUT/f$d.log"; exit 1; }
done
W="workload: tools/extract_timing.py 64 = the bench roofline pass (left batch, seed 1000, B=64)"
python3 tools/pmc_traffic.py "$(find "$OUT/fFETCH_SIZE" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT/fWRITE_SIZE" -name '*counter_collection.csv' | head -1)" "$OUT/traffic_r05.json" "$W" > /dev/null || exit 1
python3 tools/pmc_valu.py "$(find "$OUT/fSQ_INSTS_VALU" -name '*counter_collection.csv' | head -1)" "$OUT/valu_r05.json" "$W" > /dev/null || exit 1
rm -rf "$OUT/fFETCH_SIZE" "$OUT/fWRITE_SIZE" "$OUT/fSQ_INSTS_VALU"
python3 -c "
import json
m=json.load(open('$OUT/match_pmc_r05.json')); t=json.load(open('$OUT/traffic_r05.json')); v=json.load(open('$OUT/valu_r05.json'))
print({k: m[k] for k in m if 'pose' in k or 'stereo' in k or 'cand' in k})
print({k: t[k] for k in t if 'fast' in k}); print({k: v[k] for k in v if 'fast' in k})"
date
