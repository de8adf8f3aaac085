#!/bin/bash
# GPU box: bench line (no CPU baseline) for each library variant given.  usage: bash tools/ab_job.sh TAG name...
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; cd "$ROOT"; OUT=gpurun_out/$1; shift; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
for v in "$@"; do
    lib=dpg-slam_amd/lib/libdpg_$v.so; [ "$v" = base ] && lib=dpg-slam_amd/lib/libdpg.so
    DPGSLAM_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
    echo "$v $(grep -o '"icp_kernel_ms": [0-9.]*' "$OUT/$v.json") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$v.json")"
done
