#!/bin/bash
# A/B of k_pose_opt between two builds of the library: kernel stats of tools/pose_timing.py 63
# under each.  usage: bash tools/pose_ab.sh <tag> <libA.so> <libB.so>
set -o pipefail
TAG=${1:-ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for lib in "$2" "$3"; do
  n=$(basename "$lib" .so)
  ORBGPU_LIB="$lib" timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$n" -o p -- python3 tools/pose_timing.py 63 1 > "$OUT/$n.log" 2>&1 || { tail -20 "$OUT/$n.log"; exit 1; }
  echo "== $n"; grep "F=" "$OUT/$n.log"
  python3 tools/prof_csv.py "$(find "$OUT/$n" -name '*kernel_stats.csv' | head -1)" 6
done
