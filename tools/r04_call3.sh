#!/bin/bash
# round-4 call 3: global BA (device structure, config-5 8k x 10 / 16k golden fixtures), the stereo
# API change, global-BA timing device vs host structure, pipeline A/B with --stereo-batch.
set -o pipefail
TAG=${1:-r04e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stereo.py tests/test_gpu_track_local_map.py tests/test_gpu_match.py tests/test_gpu_ba.py tests/test_gpu_pnp.py tests/test_gpu_sim3.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_match.txt" 2>&1 \
  || { tail -40 "$OUT/pytest_match.txt"; exit 1; }
tail -1 "$OUT/pytest_match.txt"
timeout -k 10 300 python tools/ransac_bench.py --no-cpu > "$OUT/ransac.json" 2> "$OUT/ransac.err" || { tail -20 "$OUT/ransac.err"; exit 1; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for kd in ('pnp','sim3'):
    for k,v in d[kd].items(): print(kd, k, v['device_hyp_per_s'], v['wall_hyp_per_s'], v['wall_over_device'], v['ms_call_wall'], v['ms_call_wall_python'])" "$OUT/ransac.json"
timeout -k 10 200 python tools/ba_timing.py 30 > "$OUT/ba_timing.txt" 2>&1 || { tail -20 "$OUT/ba_timing.txt"; exit 1; }
tail -3 "$OUT/ba_timing.txt"
for h in 0 1; do
  ORBGPU_STRUCT_HOST=$h ORBGPU_BA_TIMES=1 timeout -k 10 200 python tools/gba_timing.py 2000:4 > "$OUT/gba_timing_host$h.txt" 2>&1 || { tail -20 "$OUT/gba_timing_host$h.txt"; exit 1; }
  echo "struct_host=$h"; grep "nkf\|\[ba\] call" "$OUT/gba_timing_host$h.txt" | tail -3
done
SKIP_TESTS=1 bash tools/lanes_ab.sh $TAG/lanes "--lanes 2" "--lanes 2 --stereo-batch 1" "--lanes 3 --stereo-batch 1" "ORBGPU_MATCH_STREAM_PRIO=1;--lanes 2 --stereo-batch 1" "ORBGPU_CAND_NT=256;--lanes 2 --stereo-batch 1" || exit 1
bash tools/ldlt_levels.sh $TAG/levels 2000:4 > /dev/null 2>&1 && tail -3 "$OUT/levels/levels.txt"
