#!/bin/bash
# round-4 call 2: RANSAC on the device (tests + bench leg), octree change (extraction tests),
# pipeline A/B over --lanes.
set -o pipefail
TAG=${1:-r04c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_sim3.py tests/test_gpu_extract.py tests/test_gpu_frame_ops.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 \
  || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 300 python tools/ransac_bench.py --no-cpu > "$OUT/ransac.json" 2> "$OUT/ransac.err" || { tail -20 "$OUT/ransac.err"; exit 1; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for k,v in d['pnp'].items(): print('pnp', k, v['device_hyp_per_s'], v['wall_hyp_per_s'], v['ms_call_wall'])
for k,v in d['sim3'].items(): print('sim3', k, v['device_hyp_per_s'], v['wall_hyp_per_s'], v['ms_call_wall'])" "$OUT/ransac.json"
SKIP_TESTS=1 bash tools/lanes_ab.sh $TAG/lanes 2 3
