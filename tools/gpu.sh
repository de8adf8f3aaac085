#!/bin/bash
# gpurun wrapper: stamps BUILD_GIT_SHA with the commit the pushed tree was taken from (plus
# "-dirty" when the product sources differ from it) before every call -- the tree goes to the box
# without .git, and tools/pmc_job.sh copies this stamp into the PMC record beside the source hash.
# usage: bash tools/gpu.sh TIMEOUT_S 'command'
set -u
cd "$(dirname "$0")/.."
sha=$(git rev-parse HEAD)
if ! git diff --quiet HEAD -- dpg-slam_amd/csrc include bench.py; then sha="$sha-dirty"; fi
echo "$sha" > BUILD_GIT_SHA
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
