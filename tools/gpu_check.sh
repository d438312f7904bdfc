#!/bin/bash
# One GPU-box pass: parity tests, bench line, rocprofv3 kernel stats.
# Usage (from the repo root on the box): bash tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-run}
KEXPR=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
echo "[gpu_check] pytest -m gpu" && date
if [ -n "$KEXPR" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
else
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
fi
tail -3 "$OUT/pytest_gpu.log"
echo "[gpu_check] bench" && date
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "[gpu_check] rocprofv3" && date
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline \
  > "$OUT/prof_bench.log" 2>&1 || { tail -30 "$OUT/prof_bench.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' | head -5
echo "[gpu_check] done" && date
