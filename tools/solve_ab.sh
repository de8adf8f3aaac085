#!/bin/bash
# GPU box job: the triangular solves' LDS staging A/B (tools/build/chol_bench: factor + solve and
# forward + backward alone, DPG_SOLVE_STAGE = staging region in doubles, 0 = none), the timing build's
# critical paths, then the solver parity tests and one bench line.  usage: bash tools/solve_ab.sh TAG
set -u
TAG=${1:-solve}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
for c in 4 3; do
  for R in ${RLIST:-0 2400 default 15000}; do
    if [ "$R" = default ]; then unset DPG_SOLVE_STAGE; else export DPG_SOLVE_STAGE=$R; fi
    timeout -k 10 60 tools/build/chol_bench tools/build/pairs$c.bin 40 > "$OUT/c${c}_R$R.log" 2>&1; rc=$?
    echo "config$c R=$R rc=$rc $(cat $OUT/c${c}_R$R.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
unset DPG_SOLVE_STAGE
timeout -k 10 60 tools/build/chol_bench_t tools/build/pairs4.bin 3 > "$OUT/timing4.log" 2>&1; rc=$?
echo "timing rc=$rc"; grep -E "span|critical" "$OUT/timing4.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "gn or config4 or optimize or solver or inc or reopt or slam or ranks" \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit $rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/bench.err"; exit $rc; }
