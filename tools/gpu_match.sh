#!/bin/bash
# Matcher roofline evidence: three --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ_INSTS_VALU) over the
# bench's isolated passes, the per-kernel json (profiles/match_pmc_r03.json), then the bench line
# and a kernel-stats profile of the same run.  usage: bash tools/gpu_match.sh <tag>
set -o pipefail
TAG=${1:-m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -f csv -d "$OUT/$c" -o m -- python3 "$R/bench.py" --passes-only \
    > "$OUT/$c.log" 2>&1 || { echo "$c pass failed"; tail -20 "$OUT/$c.log"; exit 1; }
done
python3 tools/pmc_match.py "$(find "$OUT/FETCH_SIZE" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT/WRITE_SIZE" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT/SQ_INSTS_VALU" -name '*counter_collection.csv' | head -1)" "$OUT/match_pmc.json" \
  "workload: bench.py --passes-only (B=64 KITTI stereo batch: 5 isolated ComputeStereoMatches + SearchByProjection(Cur,Last,7) + 16 dense 1200x1200 tiles)" > /dev/null || exit 1
cp "$OUT/match_pmc.json" profiles/match_pmc_r03.json
rm -rf "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE" "$OUT/SQ_INSTS_VALU"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
