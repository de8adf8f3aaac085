#!/bin/bash
# round-5 quick GPU job: selected GPU tests, then (optionally) the bench line.
# usage: bash tools/r5_quick.sh TAG "PYTEST_SELECTION" [bench]
set -u
TAG=${1:-q}; SEL=${2:-tests}; BENCH=${3:-}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd:$ROOT/tests
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests exit $rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench exit $rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
fi
