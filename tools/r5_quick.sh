#!/bin/bash
# round-5 quick GPU job: selected GPU tests, then (optionally) the bench line.
# usage: bash tools/r5_quick.sh TAG "PYTEST_SELECTION" [bench] [prof]   (SEL "none": no tests)
set -u
TAG=${1:-q}; SEL=${2:-tests}; BENCH=${3:-}; PROF=${4:-}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd:$ROOT/tests
cd "$ROOT"
export TMPDIR=/tmp
if [ "$SEL" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $SEL -x -v -m gpu --tb=short --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests exit $rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench exit $rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
  rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/gn_timeline.py "$OUT/prof" 2 > "$OUT/timeline.txt" 2>&1; head -40 "$OUT/timeline.txt"
fi
