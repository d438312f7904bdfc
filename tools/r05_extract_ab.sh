#!/bin/bash
# Extraction A/B (round 5): the extraction tests, then one extractor's stage timings at 128 and
# 2 images with the chained pyramid tail on / off, then the default bench line.
# usage: bash tools/r05_extract_ab.sh <tag>
set -o pipefail
TAG=${1:-r05x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_extract.txt" 2>&1 \
  || { tail -30 "$OUT/pytest_extract.txt"; exit 1; }
tail -1 "$OUT/pytest_extract.txt"
for B in 128 2; do
  for C in 0 1; do
    echo "B=$B chain=$C: $(ORBGPU_PYR_CHAIN=$C timeout -k 10 120 python tools/extract_timing.py $B 2>/dev/null | tail -1)" | tee -a "$OUT/extract_ab.txt" || exit 1
  done
done
timeout -k 10 600 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d.get('stage_ms_per_step'))" "$OUT/bench.json"
