#!/bin/bash
# GPU box job: parity tests -> full bench line (with CPU baseline) -> rocprofv3 kernel-trace stats.
# usage: bash tools/round_job.sh TAG      (each GPU step under its own time limit; stops at the first failure)
set -u
TAG=${1:-run}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
cd "$ROOT"
export TMPDIR=/tmp
(nproc; lscpu | head -20) > "$OUT/host.txt" 2>&1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests exit $rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit $rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
find "$OUT/prof" -name '*stats*' | head
