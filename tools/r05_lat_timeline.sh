#!/bin/bash
# Batch-1 frame timeline: bench.py --latency-only under rocprofv3 (kernel trace), the spacing of the
# frames' first pyramid launches, and the kernels of device-leg frames 10-12 (tools/timeline.py).
# usage: bash tools/r05_lat_timeline.sh <tag>
set -o pipefail
TAG=${1:-r05lat}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o lat -- python3 bench.py --latency-only > "$OUT/lat.json" 2> "$OUT/lat.err" || { tail -20 "$OUT/lat.err"; exit 1; }
KT=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 - "$KT" > "$OUT/pyr0_starts.txt" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
p = [r for r in rows if "k_pyr_level0" in r["Kernel_Name"]]
prev = None
for i, r in enumerate(p):
    s = int(r["Start_Timestamp"])
    print(i, r.get("Grid_Size_Z", ""), r.get("Grid_Size", ""), "" if prev is None else f"{(s - prev) / 1e3:.1f} us")
    prev = s
PY
python3 tools/prof_csv.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" 40 > "$OUT/lat_kernel_stats.txt"
FIRST=$(awk 'NR>1 && $NF=="us" && $(NF-1)+0 < 3000 {print $1; exit}' "$OUT/pyr0_starts.txt")
for k in 10 11 12; do python3 tools/timeline.py "$KT" $((FIRST + k)) 1 > "$OUT/lat_timeline_frame$k.txt"; head -1 "$OUT/lat_timeline_frame$k.txt"; done
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['latency']; print('device p50', d['p50_ms'], 'mean', d['mean_ms'], '| host path p50', d['host_path']['p50_ms'], 'mean', d['host_path']['mean_ms'])" "$OUT/lat.json"
gzip -f "$KT"; mv "$KT.gz" "$OUT/"; rm -rf "$OUT/prof"
