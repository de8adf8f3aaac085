#!/bin/bash
# GPU box job: kernel trace of the incremental workload (per-node kernel durations and gaps)
# usage: bash tools/inc_trace_job.sh TAG
set -u
TAG=${1:-inctrace}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --workload incremental --cpu-nodes 0 > "$OUT/inc.json" 2> "$OUT/inc.err"
rc=$?; echo "inc trace exit $rc"; cat "$OUT/inc.json"; exit $rc
