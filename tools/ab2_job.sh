#!/bin/bash
# GPU box: ICP parity subset, defer-cap A/B (one process), counters + clock builds at the default cap.
# usage: bash tools/ab2_job.sh TAG [caps...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; cd "$ROOT"; TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 100 --timeout-method thread > "$OUT/parity.log" 2>&1; rc=$?; tail -3 "$OUT/parity.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/icp_ab.py "$@" > "$OUT/ab.txt" 2>&1; rc=$?; cat "$OUT/ab.txt"; [ $rc -eq 0 ] || exit $rc
DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_stats.so timeout -k 10 200 python -u tools/icp_stats.py > "$OUT/stats.txt" 2>&1; rc=$?; cat "$OUT/stats.txt"; [ $rc -eq 0 ] || exit $rc
DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_timing.so timeout -k 10 200 python -u tools/icp_stats.py > "$OUT/timing.txt" 2>&1; rc=$?; cat "$OUT/timing.txt"; exit $rc
