#!/bin/bash
# PoseOptimization iteration on the GPU box: pose parity tests, then the bench line without the
# CPU baseline; prints throughput and batch-1 latency.  bash tools/pose_iter.sh <tag>
set -o pipefail
TAG=${1:-pi}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pose.py tests/test_gpu_frame_ops.py tests/test_gpu_ba_g2o_order.py \
  tests/test_gpu_track_local_map.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["value"], d["ms_per_step"], d["latency"])
PY
