#!/bin/bash
# GPU box job: parity tests, then a rocprofv3 kernel-trace profile of a short bench run.
# usage: bash tools/gpu_job.sh TAG [pytest -k expression]
# Each GPU step has its own time limit; the script stops at the first failing step.
set -u
TAG=${1:-run}
K=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
cd "$ROOT"
if [ -n "$K" ]; then
    timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "$K" > "$OUT/tests.log" 2>&1
else
    timeout -k 10 600 python -m pytest tests -x -q -m gpu > "$OUT/tests.log" 2>&1
fi
rc=$?
echo "tests exit $rc" | tee -a "$OUT/tests.log"
tail -5 "$OUT/tests.log"
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench.log" 2>&1
rc=$?
echo "bench exit $rc" | tee -a "$OUT/bench.log"
tail -3 "$OUT/bench.log"
exit $rc
