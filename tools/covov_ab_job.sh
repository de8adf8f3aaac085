#!/bin/bash
# GPU box job: batch covariance beside the GN (default) vs in stream order (DPG_COV_OVERLAP=0),
# alternated in bench.py, after the GPU tests given.  usage: bash tools/covov_ab_job.sh TAG [tests...]
set -u
OUT=gpurun_out/${1:-covov}; shift; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 500 python -u -m pytest "$@" -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
  echo "tests exit $rc"; tail -2 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2 3; do
  for m in 0 1; do
    DPG_COV_OVERLAP=$m timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${m}_$r.json 2> $OUT/b_${m}_$r.err || exit $?
    python - $OUT/b_${m}_$r.json overlap=$m <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms/step %.3f" % d["ms_per_step"], "ms/gn-iter %.4f" % d["ms_per_gn_iter"], "iters", d["gn_iterations"], "err %.12e" % d["final_error"], "icp %.3f cov %.3f" % (d["icp_kernel_ms"], d["cov_kernel_ms"]))
PY
  done
done
