#!/bin/bash
# k_pose_opt roofline evidence: one --pmc pass (SQ_INSTS_VALU, SQ_WAVES, SQ_BUSY_CYCLES) over
# tools/pose_timing.py (B=63 KITTI-shaped frames), the per-launch json -> profiles/pose_valu_r03.json,
# then the kernel stats of the same workload.  usage: bash tools/pose_pmc.sh <tag>
set -o pipefail
TAG=${1:-pp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -f csv -d "$OUT/valu" -o p -- \
  python3 tools/pose_timing.py 63 > "$OUT/valu.log" 2>&1 || { tail -20 "$OUT/valu.log"; exit 1; }
python3 tools/pmc_valu.py "$(find "$OUT/valu" -name '*counter_collection.csv' | head -1)" "$OUT/pose_valu.json" \
  "workload: tools/pose_timing.py 63 (B=63 KITTI-shaped frames, k_pose_opt<256>)" > /dev/null || exit 1
cp "$OUT/pose_valu.json" profiles/pose_valu_r03.json
timeout -k 10 90 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o p -- python3 tools/pose_timing.py 63 \
  > "$OUT/stats.log" 2>&1 || { tail -20 "$OUT/stats.log"; exit 1; }
grep "F=" "$OUT/stats.log"
python3 tools/prof_csv.py "$(find "$OUT/stats" -name '*kernel_stats.csv' | head -1)" 5 | tee "$OUT/kernel_stats.txt"
cat profiles/pose_valu_r03.json
