#!/bin/bash
# Global-BA pass on the GPU box: the LDL^T unit tests and the BA parity tests, then a rocprofv3
# kernel-stats profile of BundleAdjustment(10) at 2,000 keyframes (band and 4 laps).
# bash tools/gba_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-gc}
KEXPR=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
ARGS=(tests/test_gpu_ba_units.py tests/test_gpu_ba.py tests/test_gpu_ba_g2o_order.py tests/test_gpu_ba_sharded.py)
if [ -n "$KEXPR" ]; then ARGS+=(-k "$KEXPR"); fi
timeout -k 10 900 python -u -m pytest "${ARGS[@]}" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" "$OUT/pytest.log" | tail -60
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -f csv -o gba -- python3 tools/gba_timing.py 2000:0 2000:4 > "$OUT/gba_timing.txt" 2>&1 || { tail -20 "$OUT/gba_timing.txt"; exit 1; }
grep "nkf" "$OUT/gba_timing.txt"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv" && head -25 "$f"
exit 0
