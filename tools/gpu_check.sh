#!/bin/bash
# One GPU-box pass: parity tests, PMC passes (HBM traffic, VALU issue) of the roofline kernel,
# bench line (reads the fresh PMC files), rocprofv3 kernel stats of the bench + roofline check.
# Usage (from the repo root on the box): bash tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-run}
KEXPR=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
echo "[gpu_check] pytest -m gpu" && date
if [ -n "$KEXPR" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
else
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
fi
tail -3 "$OUT/pytest_gpu.log"
echo "[gpu_check] pmc passes" && date
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES"; do
  d=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -f csv -d "$OUT/$d" -o ex -- python3 "$R/tools/extract_timing.py" 64 \
    > "$OUT/$d.log" 2>&1 || { echo "$c pass failed"; tail -20 "$OUT/$d.log"; exit 1; }
done
W="workload: tools/extract_timing.py 64 = the bench roofline pass (left batch, seed 1000, B=64)"
python3 tools/pmc_traffic.py "$(find "$OUT/FETCH_SIZE" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT/WRITE_SIZE" -name '*counter_collection.csv' | head -1)" "$OUT/traffic.json" "$W" || exit 1
python3 tools/pmc_valu.py "$(find "$OUT/SQ_INSTS_VALU" -name '*counter_collection.csv' | head -1)" "$OUT/valu.json" "$W" || exit 1
# the box-side copy feeds this run's bench line; copy gpurun_out/<tag>/{traffic,valu}.json into
# profiles/ afterwards so the committed files (read by the round-end bench) match the kernel
cp "$OUT/traffic.json" profiles/traffic_r03.json && cp "$OUT/valu.json" profiles/valu_r03.json
echo "[gpu_check] bench" && date
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "[gpu_check] rocprofv3" && date
ORBGPU_LBA_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline \
  > "$OUT/prof_bench.log" 2>&1 || { tail -30 "$OUT/prof_bench.log"; exit 1; }
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 60 > "$OUT/kernel_stats.txt"
python3 tools/roofline_check.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" "$OUT/bench.json" | tee "$OUT/roofline_check.json"
python3 tools/timeline.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" 8 > "$OUT/timeline.txt"
echo "[gpu_check] done" && date
