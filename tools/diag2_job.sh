#!/bin/bash
# GPU box: ICP diagnostics (counter build, clock build) + one bench line.  usage: bash tools/diag2_job.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; cd "$ROOT"; OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
(nproc; lscpu) > "$OUT/host.txt" 2>&1
DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_stats.so timeout -k 10 200 python -u tools/icp_stats.py > "$OUT/stats.txt" 2>&1; rc=$?; cat "$OUT/stats.txt"; [ $rc -eq 0 ] || exit $rc
DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_timing.so timeout -k 10 200 python -u tools/icp_stats.py > "$OUT/timing.txt" 2>&1; rc=$?; cat "$OUT/timing.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?; cat "$OUT/bench.json"; exit $rc
