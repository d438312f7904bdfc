#!/bin/bash
# Round-5 GPU pass: every GPU test, smoke(), the default bench line, a rocprofv3 kernel trace of
# the bench (kernel stats, step timeline, roofline check of k_pose_opt + k_fast_cells).
# usage: bash tools/r05_check.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
if [ -z "$2" ]; then
  echo "[r05] pytest -m gpu" && date
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 \
    || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -2 "$OUT/pytest_gpu.txt"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
  cat "$OUT/smoke.txt"
fi
echo "[r05] bench" && date
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], d.get('sequence_frames_per_s'))" "$OUT/bench.json"
echo "[r05] rocprofv3" && date
ORBGPU_LBA_STREAMS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || { tail -30 "$OUT/bench_prof.err"; exit 1; }
KS=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
KT=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 tools/prof_csv.py "$KS" 60 > "$OUT/kernel_stats.txt"
python3 tools/roofline_check.py "$KT" "$OUT/bench_prof.json" | tee "$OUT/roofline_check.json"
python3 tools/timeline.py "$KT" 8 > "$OUT/timeline_step8.txt"
head -30 "$OUT/kernel_stats.txt"
rm -rf "$OUT/prof"
date
