#!/bin/bash
# Round-6 quick GPU pass: selected GPU tests (args after the tag), then the default bench line.
# usage: bash tools/r06_quick.sh <tag> [pytest selectors...]
set -o pipefail
TAG=${1:-r06q}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 \
    || { tail -40 "$OUT/pytest.txt"; exit 1; }
  tail -2 "$OUT/pytest.txt"
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d.get('value_host_io'), d['latency']['p50_ms'], d['latency']['host_path']['p50_ms'], d['local_ba'].get('single_stream'), d['global_ba'].get('value'))" "$OUT/bench.json"
fi
