#!/bin/bash
# round-5 record: the whole GPU suite, smoke(), the default bench line, a kernel-trace profile of the
# bench and its per-step timeline.  usage: bash tools/r5_final.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; OUT=$ROOT/gpurun_out/${1:-final}; mkdir -p "$OUT"; cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd:$ROOT/tests TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --tb=short --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests exit $rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke exit $rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit $rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/gn_timeline.py "$OUT/prof" 2 > "$OUT/timeline.txt" 2>&1; head -16 "$OUT/timeline.txt"
timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 > "$OUT/inc.json" 2> "$OUT/inc.err"
rc=$?; echo "inc exit $rc"; tail -c 600 "$OUT/inc.json"; [ $rc -eq 0 ] || exit $rc
