#!/bin/bash
# Round-5 A/B: extraction stage timings at 2 images per octree workgroup size, the batch-1
# latency legs, then pipeline variants (two alternating rounds).
set -o pipefail
TAG=${1:-r05ab2}
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
export TMPDIR=/tmp
for T in 256 512 1024; do
  echo "B=2 OCT_T=$T: $(ORBGPU_OCT_T=$T timeout -k 10 120 python tools/extract_timing.py 2 2>/dev/null | tail -1)" | tee -a "$OUT/oct_ab.txt" || exit 1
done
for T in 256 1024; do
  L=$(ORBGPU_OCT_T=$T timeout -k 10 300 python bench.py --latency-only 2> "$OUT/lat_err.txt") || { tail -20 "$OUT/lat_err.txt"; exit 1; }
  echo "latency OCT_T=$T: $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); l=d.get('latency', d); print(l['p50_ms'], l['mean_ms'], l['host_path']['p50_ms'], l['host_path']['mean_ms'], max(l['host_path']['frame_ms']))" "$L")" | tee -a "$OUT/lat_ab.txt"
done
bash tools/r05_pipe_ab.sh "$TAG/pipe" "base|X=0|" "blurearly|ORBGPU_BLUR_EARLY=1|" "blurside|ORBGPU_BLUR_SIDE=1|" "lanes3|X=0|--lanes 3" "xprio|ORBGPU_EXTRACT_STREAM_PRIO=1|"
