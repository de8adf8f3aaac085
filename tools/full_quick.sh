#!/bin/bash
# GPU box job: Cholesky alone (configs 3/4, factor+solve and the chord-step solves), the full GPU
# suite, smoke, one bench line and the incremental line.  usage: bash tools/full_quick.sh TAG
set -u
TAG=${1:-fq}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
for c in 4 3; do
  timeout -k 10 60 tools/build/chol_bench tools/build/pairs$c.bin 40 > "$OUT/chol$c.log" 2>&1; rc=$?
  echo "config$c rc=$rc $(cat $OUT/chol$c.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 60 tools/build/chol_bench_t tools/build/pairs4.bin 3 > "$OUT/timing4.log" 2>&1; rc=$?
echo "timing rc=$rc"; grep -E "span|critical" "$OUT/timing4.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests exit $rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke exit $rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit $rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/bench.err"; exit $rc; }
timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 > "$OUT/inc.json" 2> "$OUT/inc.err"
rc=$?; echo "inc bench exit $rc"; cat "$OUT/inc.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/inc.err"; exit $rc; }
