#!/bin/bash
# GPU box job for iteration: ICP/GN parity tests (optional -k filter), then one bench line
# without the CPU baseline.  usage: bash tools/quick_job.sh TAG [pytest -k expression]
set -u
TAG=${1:-quick}
K=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
cd "$ROOT"
if [ -n "$K" ]; then
    timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
else
    timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
fi
rc=$?; echo "tests exit $rc"; tail -4 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit $rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/bench.err"; exit $rc; }
