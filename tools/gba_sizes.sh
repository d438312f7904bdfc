#!/bin/bash
# Global BA at config-5 sizes on the GPU box: the BA parity tests, then GPU timing of
# BundleAdjustment(10) at 2,000 / 8,000 / 16,000 keyframes.  bash tools/gba_sizes.sh <tag>
set -o pipefail
TAG=${1:-gs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_g2o_order.py tests/test_gpu_ba_sharded.py -x -q \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 800 python -u tools/gba_timing.py 2000 8000 16000 2>&1 | tee "$OUT/gba_sizes.txt"
