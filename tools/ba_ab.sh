#!/bin/bash
# BA A/B between two library builds: local BA single stream (tools/ba_timing.py) and global BA at
# 2,000 keyframes, 4 laps (tools/gba_timing.py), each under rocprofv3 kernel stats, then the BA
# parity tests on the in-tree library.  usage: bash tools/ba_ab.sh <tag> <libA.so> <libB.so>
set -o pipefail
TAG=${1:-baab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for lib in "$2" "$3"; do
  n=$(basename "$lib" .so)
  export ORBGPU_LIB="$R/$lib"
  timeout -k 10 120 python3 tools/ba_timing.py 40 > "$OUT/$n.lba.txt" 2>&1 || { tail -5 "$OUT/$n.lba.txt"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$n/gba" -f csv -o gba -- python3 tools/gba_timing.py 2000:4 \
    > "$OUT/$n.gba.txt" 2>&1 || { tail -5 "$OUT/$n.gba.txt"; exit 1; }
  echo "== $n"
  cat "$OUT/$n.lba.txt"
  grep nkf "$OUT/$n.gba.txt"
  python3 tools/prof_csv.py "$(find "$OUT/$n/gba" -name '*kernel_stats.csv' | head -1)" 12
done
unset ORBGPU_LIB
timeout -k 10 700 python -u -m pytest tests/test_gpu_ba_units.py tests/test_gpu_ba.py tests/test_gpu_ba_g2o_order.py \
  tests/test_gpu_ba_sharded.py tests/test_gpu_sim3opt.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
exit $rc
