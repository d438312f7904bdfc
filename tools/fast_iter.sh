#!/bin/bash
# FAST kernel iteration on the GPU box: extraction parity tests, kernel stats, VALU pass.
# bash tools/fast_iter.sh <tag>
set -o pipefail
TAG=${1:-fi}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py -x -q \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/prof_extract.sh "$TAG" || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -f csv -d "$OUT/VALU" -o ex -- python3 tools/extract_timing.py 64 \
  > "$OUT/valu.log" 2>&1 || { tail -20 "$OUT/valu.log"; exit 1; }
python3 tools/pmc_valu.py "$(find "$OUT/VALU" -name '*counter_collection.csv' | head -1)" "$OUT/valu.json" x > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$OUT/valu.json'))['k_fast_cells']; print('k_fast_cells VALU/launch', d)"
