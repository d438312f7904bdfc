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
timeout -k 10 600 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_sim3.py tests/test_gpu_ba_units.py tests/test_gpu_ba_struct.py tests/test_gpu_ba.py tests/test_gpu_extract.py tests/test_gpu_frame_ops.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 \
  || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 300 python tools/ransac_bench.py --no-cpu > "$OUT/ransac.json" 2> "$OUT/ransac.err" || { tail -20 "$OUT/ransac.err"; exit 1; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for k,v in d['pnp'].items(): print('pnp', k, v['device_hyp_per_s'], v['wall_hyp_per_s'], v['ms_call_wall'])
for k,v in d['sim3'].items(): print('sim3', k, v['device_hyp_per_s'], v['wall_hyp_per_s'], v['ms_call_wall'])" "$OUT/ransac.json"
for v in "1 0" "0 0" "1 1"; do
  set -- $v
  ORBGPU_LDLT_ROW=$1 ORBGPU_STRUCT_HOST=$2 timeout -k 10 200 python tools/ba_timing.py 30 > "$OUT/ba_timing_row$1_host$2.txt" 2>&1 || { tail -20 "$OUT/ba_timing_row$1_host$2.txt"; exit 1; }
  echo "ldlt_row=$1 struct_host=$2"; tail -4 "$OUT/ba_timing_row$1_host$2.txt"
done
SKIP_TESTS=1 bash tools/lanes_ab.sh $TAG/lanes "--lanes 2" "--lanes 3" "--lanes 2 --reserve-cus 4"
