#!/bin/bash
# Matcher iteration on the GPU box: search/match parity tests, then the bench line without the
# CPU baseline; prints the line's headline figures.  bash tools/match_iter.sh <tag>
set -o pipefail
TAG=${1:-mi}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_search.py tests/test_gpu_track_local_map.py \
  tests/test_gpu_frame_ops.py tests/test_gpu_stereo.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
m = d["matcher_roofline"]
print(d["value"], d["ms_per_step"], d["latency"]["p50_ms"], {k: m[k]["avg_launch_ms"] for k in m if isinstance(m[k], dict)})
PY
