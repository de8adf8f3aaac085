#!/bin/bash
# GPU box diagnostics: ICP candidate counters (stats build), per-phase clock (timing build), and
# one SQ PMC pass of a bench step.  usage: bash tools/diag_job.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; cd "$ROOT"; OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_stats.so timeout -k 10 200 python -u tools/icp_stats.py > "$OUT/stats.txt" 2>&1; rc=$?; cat "$OUT/stats.txt"; [ $rc -eq 0 ] || exit $rc
DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_timing.so timeout -k 10 200 python -u tools/icp_stats.py > "$OUT/timing.txt" 2>&1; rc=$?; cat "$OUT/timing.txt"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d "$OUT/pmc1" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc1.log" 2>&1; echo "pmc1 $?"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d "$OUT/pmc2" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc2.log" 2>&1; echo "pmc2 $?"
