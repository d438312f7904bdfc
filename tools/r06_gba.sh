#!/bin/bash
# Round-6 global-BA pass: the sparse-LDL^T / global-BA GPU tests, the config-5 timing, and a
# rocprofv3 trace of one BundleAdjustment(10) (kernel stats + the last solve's launches by level).
# usage: bash tools/r06_gba.sh <tag> [notests]     (env passes through, e.g. ORBGPU_LDLT_QUAD=0)
set -o pipefail
TAG=${1:-r06gba}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_ba_units.py tests/test_gpu_ba_sharded.py -x -q --timeout 300 \
    --timeout-method thread > "$OUT/pytest_ba.txt" 2>&1 || { tail -40 "$OUT/pytest_ba.txt"; exit 1; }
  tail -1 "$OUT/pytest_ba.txt"
fi
ORBGPU_BA_TIMES=1 timeout -k 10 300 python tools/gba_timing.py 2000:4 > "$OUT/gba_timing.txt" 2>&1 || { tail -20 "$OUT/gba_timing.txt"; exit 1; }
grep nkf "$OUT/gba_timing.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o p -- python3 tools/gba_timing.py 2000:4 > "$OUT/prof.txt" 2>&1 || { tail -20 "$OUT/prof.txt"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 30 > "$OUT/gba_kernel_stats.txt"
python3 tools/ldlt_levels.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" > "$OUT/gba_ldlt_levels.txt"
head -24 "$OUT/gba_kernel_stats.txt"; tail -1 "$OUT/gba_ldlt_levels.txt"
rm -rf "$OUT/prof"
