#!/bin/bash
# round-4 combined pass: call 2 (RANSAC / octree / row LDL^T / device structure tests + timings +
# pipeline A/B) then call 3 (stereo API, global BA timings, sharded + config-5 golden tests).
set -o pipefail
TAG=${1:-r04f}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
bash tools/r04_call2.sh "$TAG/c2" && bash tools/r04_call3.sh "$TAG/c3"
