#!/bin/bash
# Round-5 A/B 3: kernel trace of one extractor at 2 images (octree latency), then the tracking
# lane's local-search variants in the pipeline (two alternating rounds).
set -o pipefail
TAG=${1:-r05ab3}
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/prof2" -o ex -- python3 tools/extract_timing.py 2 > /dev/null 2>&1 || exit 1
KT=$(find "$OUT/prof2" -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py "$KT" 8 > "$OUT/timeline_B2.txt"; cat "$OUT/timeline_B2.txt"; rm -rf "$OUT/prof2"
bash tools/r05_pipe_ab.sh "$TAG/pipe" "base|X=0|" "cand256|ORBGPU_CAND_NT=256|" "nostage|ORBGPU_CAND_LOCAL_STAGE=0|" "sel512|ORBGPU_SELECT_LOCAL_NT=512|" "posewide|ORBGPU_POSE_WIDE_MAX=8|"
