#!/bin/bash
# GPU box job: the Cholesky alone (tools/build/chol_bench) on configs 2-4 patterns, fused DAG path and
# level-scheduled path (DPG_CHOL_LEVELS=1); then the GN parity tests.  usage: bash tools/chol_ab.sh TAG [pytest -k]
set -u
TAG=${1:-chol}
K=${2:-gn or config4 or optimize}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
for c in 2 3 4; do
  timeout -k 10 60 tools/build/chol_bench tools/build/pairs$c.bin 20 > "$OUT/fused$c.log" 2>&1; rc=$?
  echo "fused config$c rc=$rc $(cat $OUT/fused$c.log)"; [ $rc -eq 0 ] || exit $rc
done
DPG_CHOL_LEVELS=1 timeout -k 10 60 tools/build/chol_bench tools/build/pairs4.bin 20 > "$OUT/levels4.log" 2>&1; rc=$?
echo "levels config4 rc=$rc $(cat $OUT/levels4.log)"; [ $rc -eq 0 ] || exit $rc
DPG_CHOL_SINGLE_BUFFER=1 timeout -k 10 60 tools/build/chol_bench tools/build/pairs4.bin 20 > "$OUT/single4.log" 2>&1; rc=$?
echo "single-buffer config4 rc=$rc $(cat $OUT/single4.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/build/chol_bench_t tools/build/pairs4.bin 3 > "$OUT/timing4.log" 2>&1; rc=$?
echo "timing rc=$rc"; grep -E "span|critical" "$OUT/timing4.log"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    tools/build/chol_bench tools/build/pairs4.bin 5 > "$OUT/prof.log" 2>&1; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ -n "$K" ] || exit 0
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 "$OUT/tests.log"; exit $rc
