#!/bin/bash
# PoseOptimization on the GPU box: section timers (instrumented build), then the VALU (PMC) and
# duration (kernel stats) of k_pose_opt on a batch of 63 KITTI-shaped frames.
# usage: bash tools/pose_check.sh <tag>   (needs `make -C c_orb_slam_amd/csrc prof` beforehand)
set -o pipefail
TAG=${1:-pc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
ORBGPU_LIB=build/liborbslam_gpu_prof.so timeout -k 10 120 python3 tools/pose_prof.py > "$OUT/pose_prof.txt" 2>&1 || { tail "$OUT/pose_prof.txt"; exit 1; }
cat "$OUT/pose_prof.txt"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -f csv -d "$OUT/VALU" -o p -- python3 tools/pose_timing.py 63 \
  > "$OUT/valu.log" 2>&1 || { tail -20 "$OUT/valu.log"; exit 1; }
python3 tools/pmc_valu.py "$(find "$OUT/VALU" -name '*counter_collection.csv' | head -1)" "$OUT/pose_valu.json" \
  "workload: tools/pose_timing.py 63 (63 frames x pose_problem N=2000)" || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o p -- python3 tools/pose_timing.py 63 > "$OUT/time.log" 2>&1 || { tail -20 "$OUT/time.log"; exit 1; }
cat "$OUT/time.log"
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 10
