#!/bin/bash
# Dense/sparse LDL^T rework: unit + BA parity tests, local BA (column-owner vs panel kernel),
# global BA (rolled vs unrolled panel kernels) timings and per-level launches.
# usage: bash tools/r04_ldlt.sh <tag>
set -o pipefail
TAG=${1:-r04l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
# (phase microbenchmark: tools/micro/ldlt_col.hip)
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba_units.py tests/test_gpu_ba.py tests/test_gpu_ba_g2o_order.py tests/test_gpu_ba_struct.py tests/test_gpu_pnp.py tests/test_gpu_sim3.py tests/test_gpu_stereo.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_ba.txt" 2>&1 \
  || { tail -40 "$OUT/pytest_ba.txt"; exit 1; }
tail -1 "$OUT/pytest_ba.txt"
timeout -k 10 300 python tools/ransac_bench.py --no-cpu > "$OUT/ransac.json" 2> "$OUT/ransac.err" || { tail -20 "$OUT/ransac.err"; exit 1; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for kd in ('pnp','sim3'):
    for k,v in d[kd].items(): print(kd, k, v['device_hyp_per_s'], v['wall_hyp_per_s'], v['wall_over_device'], v['ms_call_wall'])" "$OUT/ransac.json"
for v in reg 2d; do
  ORBGPU_LDLT_DENSE=$v timeout -k 10 200 python tools/ba_timing.py 30 > "$OUT/ba_timing_$v.txt" 2>&1 || { tail -20 "$OUT/ba_timing_$v.txt"; exit 1; }
  echo "dense=$v"; tail -2 "$OUT/ba_timing_$v.txt"
done
for v in 0 1; do
  ORBGPU_LDLT_PROW=$v ORBGPU_BA_TIMES=1 timeout -k 10 200 python tools/gba_timing.py 2000:4 > "$OUT/gba_timing_roll$v.txt" 2>&1 || { tail -20 "$OUT/gba_timing_roll$v.txt"; exit 1; }
  echo "prow1wave=$v"; grep "nkf" "$OUT/gba_timing_roll$v.txt"
done
bash tools/ldlt_levels.sh $TAG/levels 2000:4 > /dev/null 2>&1 && tail -8 "$OUT/levels/levels.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/lba" -o p -- python3 tools/ba_timing.py 20 > "$OUT/lba_prof.txt" 2>&1 || { tail -20 "$OUT/lba_prof.txt"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/lba" -name '*kernel_stats.csv' | head -1)" 16 | tee "$OUT/lba_kernel_stats.txt"
rm -rf "$OUT/lba"
