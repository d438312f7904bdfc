#!/bin/bash
# round-4 call 4: config-5 sharded / large parity (8k x optimize(10), 16k x 1 golden fixtures)
set -o pipefail
TAG=${1:-r04f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_ba_sharded.py -x -v --timeout 900 --timeout-method thread > "$OUT/pytest_sharded.txt" 2>&1 \
  || { tail -40 "$OUT/pytest_sharded.txt"; exit 1; }
tail -12 "$OUT/pytest_sharded.txt"
