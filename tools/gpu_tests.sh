#!/bin/bash
# Selected GPU test files on the box: bash tools/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/$TAG"
cd "$R" || exit 1
timeout -k 10 700 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > "gpurun_out/$TAG/pytest.log" 2>&1
rc=$?
tail -40 "gpurun_out/$TAG/pytest.log"
exit $rc
