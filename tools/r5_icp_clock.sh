#!/bin/bash
# ICP per-phase clock (timing build), counters (stats build) and the in-step penalty probe on config 4
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; OUT=$ROOT/gpurun_out/${1:-icpclk}; mkdir -p "$OUT"; cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
L=$ROOT/dpg-slam_amd/lib
DPGSLAM_LIB=$L/libdpg_timing.so timeout -k 10 120 python tools/icp_stats.py > "$OUT/clock.txt" 2>&1 || exit 1
cat "$OUT/clock.txt"
DPGSLAM_LIB=$L/libdpg_stats.so timeout -k 10 120 python tools/icp_stats.py > "$OUT/stats.txt" 2>&1 || exit 1
cat "$OUT/stats.txt"
AB_ROUNDS=5 timeout -k 10 300 python tools/icp_context_probe.py > "$OUT/context.txt" 2>&1 || exit 1
cat "$OUT/context.txt"
