#!/bin/bash
# A/B of the bench pipeline: extraction tests, then --pipeline-only lines for each --lanes value
# (two runs each, interleaved).  usage: bash tools/lanes_ab.sh <tag> [lanes...]
set -o pipefail
TAG=${1:-lanes}
shift
LANES=${@:-2 3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || { timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_frame_ops.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_extract.txt" 2>&1 || { tail -30 "$OUT/pytest_extract.txt"; exit 1; }; }
[ -n "$SKIP_TESTS" ] || tail -1 "$OUT/pytest_extract.txt"
for rep in 1 2; do
  for l in $LANES; do
    timeout -k 10 300 python bench.py --pipeline-only --no-cpu-baseline --steps 80 --lanes $l > "$OUT/pipe_l${l}_$rep.json" 2> "$OUT/pipe_l${l}_$rep.err" \
      || { tail -20 "$OUT/pipe_l${l}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('lanes', sys.argv[2], d['value'], d['ms_per_step'], d['phase_ms_per_step'], d['stage_ms_per_step_by_image'])" "$OUT/pipe_l${l}_$rep.json" $l
  done
done
