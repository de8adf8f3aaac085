#!/bin/bash
# the Cholesky's critical path on the config-4 pattern: per-front / per-panel in-kernel stamps
# (tools/build/chol_bench_t) and the plain build's times.  usage: bash tools/r5_chol_t.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; OUT=$ROOT/gpurun_out/${1:-cholt}; mkdir -p "$OUT"; cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
python tools/make_pairs.py config4 "$OUT/pairs.bin" || exit 1
timeout -k 10 60 tools/build/chol_bench "$OUT/pairs.bin" 20 > "$OUT/chol.log" 2>&1 || exit 1
tail -1 "$OUT/chol.log"
timeout -k 10 60 tools/build/chol_bench_t "$OUT/pairs.bin" 3 > "$OUT/timing.log" 2>&1 || exit 1
grep -E "span|critical" "$OUT/timing.log"
