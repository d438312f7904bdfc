#!/bin/bash
# BA checkpoint: every BA GPU test, local-BA and global-BA timings (one GPU).
# usage: bash tools/r05_ba_check.sh <tag>
set -o pipefail
TAG=${1:-r05bac}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ba_units.py tests/test_gpu_ba.py tests/test_gpu_ba_g2o_order.py tests/test_gpu_ba_struct.py tests/test_gpu_ba_sharded.py tests/test_gpu_sim3opt.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_ba.txt" 2>&1 \
  || { tail -40 "$OUT/pytest_ba.txt"; exit 1; }
tail -1 "$OUT/pytest_ba.txt"
ORBGPU_BA_TIMES=1 timeout -k 10 200 python tools/ba_timing.py 30 > "$OUT/ba_timing.txt" 2>&1 || { tail -20 "$OUT/ba_timing.txt"; exit 1; }
tail -2 "$OUT/ba_timing.txt"
timeout -k 10 300 python tools/gba_timing.py 2000:4 > "$OUT/gba_timing.txt" 2>&1 || { tail -20 "$OUT/gba_timing.txt"; exit 1; }
grep nkf "$OUT/gba_timing.txt"
