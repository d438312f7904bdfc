#!/bin/bash
# PMC passes over ONE extractor on a batch of 64 KITTI-shaped images (tools/extract_timing.py),
# one rocprofv3 --pmc run per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage on the GPU box, from the repo root: bash tools/pmc_extract.sh <tag>
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/extract_timing.py 64 > "$OUT/warm.log" 2>&1 || { tail -20 "$OUT/warm.log"; exit 1; }
cat "$OUT/warm.log"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  echo "[pmc] pass $i: $grp" && date
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$OUT/p$i" -o ex -- python3 "$R/tools/extract_timing.py" 64 \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
  f=$(find "$OUT/p$i" -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && python3 tools/pmc_agg.py "$f" k_ > "$OUT/p$i.agg.txt" && cat "$OUT/p$i.agg.txt"
done
echo "[pmc] done" && date
