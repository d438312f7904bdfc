#!/bin/bash
# Sharded factorisation of the global BA: in-process multi-rank parity tests + the BA suites.
# usage: bash tools/r04_dist.sh <tag>
set -o pipefail
TAG=${1:-r04d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ba_sharded.py -k "sharded or factorisation" -x -v --timeout 600 --timeout-method thread > "$OUT/pytest_sharded.txt" 2>&1 \
  || { tail -60 "$OUT/pytest_sharded.txt"; exit 1; }
grep -E "PASS|FAIL|passed|failed" "$OUT/pytest_sharded.txt" | tail -30
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba_units.py tests/test_gpu_ba.py tests/test_gpu_ba_g2o_order.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_ba.txt" 2>&1 \
  || { tail -40 "$OUT/pytest_ba.txt"; exit 1; }
tail -1 "$OUT/pytest_ba.txt"
ORBGPU_BA_TIMES=1 timeout -k 10 200 python tools/gba_timing.py 2000:4 > "$OUT/gba_timing.txt" 2>&1 || { tail -20 "$OUT/gba_timing.txt"; exit 1; }
grep "nkf" "$OUT/gba_timing.txt"
