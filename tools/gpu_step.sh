#!/bin/bash
# One GPU-box pass for the tracking lane: parity (match/stereo/pose/sim3opt), bench line,
# rocprofv3 kernel trace of the bench (timeline), k_pose_opt section timers (prof build).
# usage: bash tools/gpu_step.sh <tag>
set -o pipefail
TAG=${1:-st}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_stereo.py tests/test_gpu_pose.py \
  tests/test_gpu_search.py tests/test_gpu_frame_ops.py tests/test_gpu_sim3opt.py -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline \
  > "$OUT/prof_bench.log" 2>&1 || { tail -30 "$OUT/prof_bench.log"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 40 > "$OUT/kernel_stats.txt"
python3 tools/timeline.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" 8 > "$OUT/timeline.txt"
cat "$OUT/timeline.txt"
ORBGPU_LIB=build/liborbslam_gpu_prof.so timeout -k 10 120 python3 tools/pose_prof.py > "$OUT/pose_prof.txt" 2>&1 || { tail "$OUT/pose_prof.txt"; exit 1; }
cat "$OUT/pose_prof.txt"
