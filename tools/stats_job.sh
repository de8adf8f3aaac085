#!/bin/bash
# GPU box: ICP candidate counters (stats build) only.  usage: bash tools/stats_job.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; cd "$ROOT"; OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_stats.so timeout -k 10 200 python -u tools/icp_stats.py > "$OUT/stats.txt" 2>&1; rc=$?; cat "$OUT/stats.txt"; exit $rc
