#!/bin/bash
# GPU box job: native (dpg_gn_run) vs Python GN loop in bench.py, alternated, then the solver tests.
set -u
OUT=gpurun_out/${1:-gnrun}; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests exit $rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for m in python native; do
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --gn-loop $m > $OUT/b_${m}_$r.json 2> $OUT/b_${m}_$r.err || exit $?
    python - $OUT/b_${m}_$r.json $m <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s=d
print(sys.argv[2], "ms/step %.3f" % d["ms_per_step"], "ms/gn-iter %.4f" % s["ms_per_gn_iter"], "iters", s["gn_iterations"], "err %.9e" % s["final_error"], "icp %.3f" % s["icp_kernel_ms"])
PY
  done
done
