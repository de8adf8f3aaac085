#!/bin/bash
# GPU box job (round 4): selected GPU test files, then (BENCH=1) bench lines.
# usage: bash tools/r4_job.sh TAG [test files...]
#   BENCH=1   N=1 bench (both ICP schedules, interleaved) + a 2-virtual-device bench line
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
  echo "tests exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -40
  [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $OUT/tests.log | tail -80; exit $rc; }
fi
if [ "${BENCH:-0}" = 1 ]; then
  for r in 1 2; do
    for s in measured caller; do
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --schedule $s > $OUT/b_${s}_$r.json 2> $OUT/b_${s}_$r.err || { echo "bench $s failed"; tail -20 $OUT/b_${s}_$r.err; exit 1; }
      python - $OUT/b_${s}_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "ms/step %.3f icp %.3f gn/iter %.4f iters %.1f fact %.1f" % (d["ms_per_step"], d["icp_kernel_ms"], d["ms_per_gn_iter"], d["gn_iterations"], d["gn_factorizations"]))
PY
    done
  done
  timeout -k 10 300 python -u bench.py --virtual 2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/b_virtual2.json 2> $OUT/b_virtual2.err || { echo "virtual bench failed"; tail -20 $OUT/b_virtual2.err; exit 1; }
  tail -c 1500 $OUT/b_virtual2.json
fi
