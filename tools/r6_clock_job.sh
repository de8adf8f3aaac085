#!/bin/bash
# GPU box job (round 6): the ICP kernel in bench.py's step placement against back to back, plain
# and with the per-phase clock build (tools/icp_step_clock.py).  usage: bash tools/r6_clock_job.sh TAG
set -u
TAG=${1:-clock}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u tools/icp_step_clock.py > $OUT/plain.txt 2>&1; rc=$?; cat $OUT/plain.txt; [ $rc -eq 0 ] || exit $rc
DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_timing.so timeout -k 10 300 python -u tools/icp_step_clock.py > $OUT/timing.txt 2>&1
rc=$?; cat $OUT/timing.txt; exit $rc
