#!/bin/bash
# A/B of k_ldlt_panel's roles per workgroup on the config-5 global BA timing (one GPU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06pab}
mkdir -p "$OUT"; cd "$R" || exit 1
for v in 3 1 7 3; do
  echo "roles $v" >> "$OUT/ab.txt"
  ORBGPU_LDLT_PANEL_ROLES=$v timeout -k 10 300 python tools/gba_timing.py 2000:4 >> "$OUT/ab.txt" 2>&1 || exit 1
done
echo "legacy panels" >> "$OUT/ab.txt"
ORBGPU_LDLT_PANEL=0 timeout -k 10 300 python tools/gba_timing.py 2000:4 >> "$OUT/ab.txt" 2>&1 || exit 1
cat "$OUT/ab.txt"
