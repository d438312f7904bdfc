#!/bin/bash
# Instruction-cache and wave-state counters of the global-BA sparse LDL^T kernels (one
# BundleAdjustment at 2,000 KFs / 4 laps) and of local BA's dense k_ldlt_reg (config 4).
# usage: bash tools/ldlt_icache.sh <tag>
set -o pipefail
TAG=${1:-lic}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES \
  --kernel-trace -f csv -d "$OUT/gic" -o p -- python3 tools/gba_timing.py 2000:4 > "$OUT/gic.log" 2>&1 || { tail -20 "$OUT/gic.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES \
  --kernel-trace -f csv -d "$OUT/gw" -o p -- python3 tools/gba_timing.py 2000:4 > "$OUT/gw.log" 2>&1 || { tail -20 "$OUT/gw.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES \
  --kernel-trace -f csv -d "$OUT/lic" -o p -- python3 tools/ba_timing.py 5 > "$OUT/lic.log" 2>&1 || { tail -20 "$OUT/lic.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES \
  --kernel-trace -f csv -d "$OUT/lw" -o p -- python3 tools/ba_timing.py 5 > "$OUT/lw.log" 2>&1 || { tail -20 "$OUT/lw.log"; exit 1; }
for d in gic gw lic lw; do
  f=$(find "$OUT/$d" -name '*counter_collection.csv' | head -1)
  echo "== $d"; python3 tools/pmc_agg.py "$f" k_ldlt | tee "$OUT/$d.txt"
  rm -rf "$OUT/$d"
done
