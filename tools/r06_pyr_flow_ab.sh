#!/bin/bash
# The one-launch pyramid (k_pyr_flow) vs the launch per level (ORBGPU_PYR_FLOW=0): extraction and
# matcher GPU tests, then the pipeline-only bench interleaved, and the extractor's stage times.
# usage: bash tools/r06_pyr_flow_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06pf}
mkdir -p "$OUT"; cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_gpu_match.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 \
  || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
for rep in 1 2; do
  for f in 1 0; do
    echo "flow $f" >> "$OUT/ab.txt"
    ORBGPU_PYR_FLOW=$f timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline --steps 60 > "$OUT/run.json" 2>> "$OUT/err.txt" || { tail -20 "$OUT/err.txt"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d.get('stage_ms_per_step'))" "$OUT/run.json" >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
