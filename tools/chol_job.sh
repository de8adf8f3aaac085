#!/bin/bash
# GPU box job: time the Cholesky alone on the config4 pattern (tools/chol_bench) under rocprofv3.
# usage: bash tools/chol_job.sh TAG
set -u
TAG=${1:-chol}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
python tools/make_pairs.py config4 "$OUT/pairs.bin" || exit 1
export TMPDIR=/tmp
timeout -k 10 120 tools/build/chol_bench "$OUT/pairs.bin" 20 > "$OUT/chol.log" 2>&1
rc=$?
cat "$OUT/chol.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    tools/build/chol_bench "$OUT/pairs.bin" 5 > "$OUT/chol_prof.log" 2>&1
timeout -k 10 120 tools/build/chol_bench_t "$OUT/pairs.bin" 1 > "$OUT/chol_timing.log" 2>&1
