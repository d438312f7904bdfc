#!/bin/bash
# Extraction loop on the GPU box: parity tests, kernel stats, FETCH/WRITE passes.  bash tools/quick_extract.sh <tag>
set -o pipefail
TAG=${1:-qe}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_gpu_match.py -x -q \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash tools/prof_extract.sh "$TAG" || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -f csv -d "$OUT/$c" -o ex -- python3 "$R/tools/extract_timing.py" 64 \
    > "$OUT/$c.log" 2>&1 || { echo "$c pass failed"; tail -20 "$OUT/$c.log"; exit 1; }
  python3 tools/pmc_agg.py "$(find "$OUT/$c" -name '*counter_collection.csv' | head -1)" k_
done
