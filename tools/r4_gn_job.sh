#!/bin/bash
# GPU box job (round 4): GN-path GPU tests, two bench lines, the covariance workgroup A/B on the step.
# usage: bash tools/r4_gn_job.sh TAG [test files...]
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
  echo "tests exit $rc"; grep -E "passed|failed" $OUT/tests.log | tail -3
  [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $OUT/tests.log | tail -80; exit $rc; }
fi
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b_$r.json 2> $OUT/b_$r.err || { echo "bench failed"; tail -20 $OUT/b_$r.err; exit 1; }
  python - $OUT/b_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "ms/step %.3f icp %.3f gn/iter %.4f iters %.1f fact %.1f" % (d["ms_per_step"], d["icp_kernel_ms"], d["ms_per_gn_iter"], d["gn_iterations"], d["gn_factorizations"]))
PY
done
if [ -n "${COVAB:-}" ]; then
  AB_ROUNDS=4 timeout -k 10 300 python -u tools/step_ab.py cov_workgroups $COVAB > $OUT/covab.txt 2>&1; rc=$?; cat $OUT/covab.txt; exit $rc
fi
