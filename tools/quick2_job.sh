#!/bin/bash
# GPU box: a pytest subset (-m gpu), verbose, bounded.  usage: bash tools/quick2_job.sh TAG "pytest args..."
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; cd "$ROOT"; TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread "$@" > "$OUT/tests.log" 2>&1
rc=$?; tail -25 "$OUT/tests.log"; exit $rc
