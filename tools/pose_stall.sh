#!/bin/bash
# Where k_pose_opt's wave-cycles go, per library build: the SQ wave-state counters
# (WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY, MI355X_MICROARCH.md), the
# instruction-cache counters (separate --pmc passes) and the kernel stats of
# tools/pose_timing.py 63.  usage: bash tools/pose_stall.sh <tag> [lib.so ...]
set -o pipefail
TAG=${1:-ps}
shift
LIBS=("$@")
[ ${#LIBS[@]} -eq 0 ] && LIBS=(c_orb_slam_amd/liborbslam_gpu.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for lib in "${LIBS[@]}"; do
  n=$(basename "$lib" .so)
  export ORBGPU_LIB="$R/$lib"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES \
    --kernel-trace -f csv -d "$OUT/$n/wait" -o p -- python3 tools/pose_timing.py 63 > "$OUT/$n.wait.log" 2>&1 || { tail -20 "$OUT/$n.wait.log"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
    --kernel-trace -f csv -d "$OUT/$n/ic" -o p -- python3 tools/pose_timing.py 63 > "$OUT/$n.ic.log" 2>&1 || { tail -20 "$OUT/$n.ic.log"; exit 1; }
  timeout -k 10 90 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$n/stats" -o p -- python3 tools/pose_timing.py 63 \
    > "$OUT/$n.stats.log" 2>&1 || { tail -20 "$OUT/$n.stats.log"; exit 1; }
  echo "== $n"
  grep "F=" "$OUT/$n.stats.log"
  python3 tools/pmc_agg.py "$(find "$OUT/$n/wait" -name '*counter_collection.csv' | head -1)" k_pose_opt
  python3 tools/pmc_agg.py "$(find "$OUT/$n/ic" -name '*counter_collection.csv' | head -1)" k_pose_opt
  python3 tools/prof_csv.py "$(find "$OUT/$n/stats" -name '*kernel_stats.csv' | head -1)" 3
done
