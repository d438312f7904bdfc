#!/bin/bash
# Round-end evidence on the GPU box: every GPU test, smoke(), the default bench line, and a
# rocprofv3 kernel-stats profile of the bench command (CPU baselines off: the same kernels).
# usage: bash tools/final_check.sh <tag>     (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 \
  || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
cat "$OUT/smoke.txt"
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['frac'])" "$OUT/bench.json"
ORBGPU_LBA_STREAMS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || { tail -30 "$OUT/bench_prof.err"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 40 > "$OUT/kernel_stats.txt"
cp "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv"
rm -rf "$OUT/prof"
head -25 "$OUT/kernel_stats.txt"
