#!/bin/bash
# Local BA single-stream profile: timing, a kernel trace of tools/ba_timing.py with the last call's
# timeline (tools/lba_timeline.py) and per-kernel stats.
# usage: bash tools/r05_lba.sh <tag>
set -o pipefail
TAG=${1:-r05lba}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
if [ "${LBA_TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ba_units.py tests/test_gpu_ba.py tests/test_gpu_ba_g2o_order.py tests/test_gpu_ba_struct.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_ba.txt" 2>&1 \
    || { tail -40 "$OUT/pytest_ba.txt"; exit 1; }
  tail -1 "$OUT/pytest_ba.txt"
fi
ORBGPU_BA_TIMES=1 timeout -k 10 200 python tools/ba_timing.py 30 > "$OUT/ba_timing.txt" 2>&1 || { tail -20 "$OUT/ba_timing.txt"; exit 1; }
tail -3 "$OUT/ba_timing.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d "$OUT/lba" -o p -- python3 tools/ba_timing.py 10 > "$OUT/lba_prof.txt" 2>&1 || { tail -20 "$OUT/lba_prof.txt"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/lba" -name '*kernel_stats.csv' | head -1)" 30 > "$OUT/lba_kernel_stats.txt"
python3 tools/lba_timeline.py "$(find "$OUT/lba" -name '*kernel_trace.csv' | head -1)" "$(find "$OUT/lba" -name '*memory_copy_trace.csv' | head -1)" > "$OUT/lba_timeline.txt"
head -20 "$OUT/lba_kernel_stats.txt"; tail -1 "$OUT/lba_timeline.txt"
rm -rf "$OUT/lba"
