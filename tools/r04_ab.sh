#!/bin/bash
# Round-4 A/B pass (no tests): RANSAC wall vs device, local-BA dense solver variants, global-BA
# structure device vs host + per-level LDL^T launches, pipeline variants (lanes, CU reserve,
# stereo batch, matcher stream priority).  usage: bash tools/r04_ab.sh <tag>
set -o pipefail
TAG=${1:-r04b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
echo "[ab] ransac" && date
timeout -k 10 300 python tools/ransac_bench.py --no-cpu > "$OUT/ransac.json" 2> "$OUT/ransac.err" || { tail -20 "$OUT/ransac.err"; exit 1; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for kd in ('pnp','sim3'):
    for k,v in d[kd].items(): print(kd, k, v['device_hyp_per_s'], v['wall_hyp_per_s'], v['wall_over_device'], v['ms_call_wall'], v.get('ms_call_wall_python'))" "$OUT/ransac.json"
echo "[ab] local BA" && date
for v in 0 1; do
  ORBGPU_LDLT_ROW=$v timeout -k 10 200 python tools/ba_timing.py 30 > "$OUT/ba_timing_row$v.txt" 2>&1 || { tail -20 "$OUT/ba_timing_row$v.txt"; exit 1; }
  echo "ldlt_row=$v"; tail -3 "$OUT/ba_timing_row$v.txt"
done
echo "[ab] global BA" && date
for h in 0 1; do
  ORBGPU_STRUCT_HOST=$h ORBGPU_BA_TIMES=1 timeout -k 10 200 python tools/gba_timing.py 2000:4 > "$OUT/gba_timing_host$h.txt" 2>&1 || { tail -20 "$OUT/gba_timing_host$h.txt"; exit 1; }
  echo "struct_host=$h"; grep "nkf\|\[ba\] call\|structure" "$OUT/gba_timing_host$h.txt" | tail -8
done
bash tools/ldlt_levels.sh $TAG/levels 2000:4 > /dev/null 2>&1 && tail -40 "$OUT/levels/levels.txt"
echo "[ab] pipeline" && date
SKIP_TESTS=1 bash tools/lanes_ab.sh $TAG/lanes "--lanes 2" "--lanes 3" "--lanes 2 --reserve-cus 4" "--lanes 2 --stereo-batch 1" "ORBGPU_MATCH_STREAM_PRIO=1;--lanes 2" || exit 1
date
