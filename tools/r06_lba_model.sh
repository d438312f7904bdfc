#!/bin/bash
# Multi-GPU cost model of config 4 (LocalBundleAdjustment keyframe-block sharded): kernel traces
# of 1, 2, 4, 8 in-process ranks of one call, then tools/gba_rank_model.py (device time only:
# the host-driven LM's round trips per trial are outside it).
# usage: bash tools/r06_lba_model.sh <tag>
set -o pipefail
TAG=${1:-r06lba}
R0=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R0/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R0" || exit 1
export TMPDIR=/tmp
ARGS=""
for R in 1 2 4 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/prof$R" -o lba -- python3 tools/gba_rank_run.py $R 0:0 local > "$OUT/run$R.txt" 2> "$OUT/run$R.err" || { tail -20 "$OUT/run$R.err"; exit 1; }
  cat "$OUT/run$R.txt"
  KT=$(find "$OUT/prof$R" -name '*kernel_trace.csv' | head -1)
  cp "$KT" "$OUT/trace$R.csv"
  rm -rf "$OUT/prof$R"
  XD=$(sed -n 's/.*exchange_doubles_per_trial \([0-9]*\).*/\1/p' "$OUT/run$R.txt")
  TR=$(sed -n 's/.* trials \([0-9]*\) .*/\1/p' "$OUT/run$R.txt")
  ARGS="$ARGS $R:$OUT/trace$R.csv:$XD:$TR"
done
python3 tools/gba_rank_model.py 1 $ARGS | tee "$OUT/model.txt"
gzip -f "$OUT"/trace*.csv
