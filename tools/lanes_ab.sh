#!/bin/bash
# A/B of the bench pipeline: --pipeline-only lines for each variant ("[ENV=val ...;]bench args"),
# two runs each, interleaved.  usage: bash tools/lanes_ab.sh <tag> "<args A>" "<args B>" ...
set -o pipefail
TAG=${1:-lanes}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || { timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_frame_ops.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_extract.txt" 2>&1 || { tail -30 "$OUT/pytest_extract.txt"; exit 1; }; }
[ -n "$SKIP_TESTS" ] || tail -1 "$OUT/pytest_extract.txt"
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    # a variant is "[ENV=val ...;]bench args"
    envs=""; args="$v"
    case "$v" in *";"*) envs="${v%%;*}"; args="${v#*;}";; esac
    timeout -k 10 300 env $envs python bench.py --pipeline-only --no-cpu-baseline --steps 80 $args > "$OUT/pipe_v${i}_$rep.json" 2> "$OUT/pipe_v${i}_$rep.err" \
      || { tail -20 "$OUT/pipe_v${i}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(repr(sys.argv[2]), d['value'], d['ms_per_step'], d['phase_ms_per_step'], {k: {s: round(x, 3) for s, x in v.items()} for k, v in d['stage_ms_per_step_by_image'].items()})" "$OUT/pipe_v${i}_$rep.json" "$v"
  done
done
